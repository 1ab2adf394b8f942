"""Native step glue: the small tensor plumbing of a model's forward / backward that would otherwise
launch ATen kernels, each as ONE launch of the framework's own kernels
(``csrc/kernels/elementwise.hip``), with a plain PyTorch reference for CPU tensors.

* :func:`first_token` -- ``h[:, 0]`` of a [B, S, H] sequence (BERT's pooler input).  Backward writes the
  whole [B, S, H] gradient in one pass (the row of position 0, zeros elsewhere) instead of autograd's
  select_backward (zero fill + copy).
* :func:`embedding_residual` -- BERT's ``position_embeddings[:S] + token_type_embeddings[0]``, the
  residual its embedding LayerNorm adds.  Backward folds the incoming [1, S, H] gradient straight into
  the two parameters' gradient-arena slots (rows 0..S-1 of the position table; the column sums over S
  into token type 0's row) -- no slice / select backward, no broadcast sum, no AccumulateGrad adds.

* :func:`prepend_token_add` -- ViT's ``cat([cls_token.expand(B), patches], 1) + position_embeddings``
  in one pass (``ddl_seq_prepend_add``).  Backward: the patch tokens' gradient as one strided copy, the
  position table's as one column-sum pass over the batch, the class token's from that sum's first row --
  straight into the parameters' gradient-arena slots when they have them.

Reference: the model files these replace call sites in (``models/bert.py``, ``models/vit.py``; HF's
``BertEmbeddings`` / ``BertPooler`` / ``ViTEmbeddings``, which the CPU oracle tests compare against).
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import call, dcode, grad_ready, grad_sink, p
from . import _native_elementwise as E


class _FirstToken(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        B, S, H = h.shape
        h = h.contiguous()
        out = torch.empty(B, H, dtype=h.dtype, device=h.device)
        E.copy2d(out, h, H, B, H, S * H, B, H)
        ctx.shape = (B, S, H)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, S, H = ctx.shape
        dout = dout.contiguous()
        dh = torch.empty(B, S, H, dtype=dout.dtype, device=dout.device)
        E.copy2d(dh, dout, S * H, B, S * H, H, B, H)      # row b: [dout[b] | zeros]
        return dh


def first_token(h: torch.Tensor) -> torch.Tensor:
    """``h[:, 0]`` (contiguous [B, H])."""
    if h.dim() == 3 and h.dtype in (torch.bfloat16, torch.float32) and _lib.use_native(h):
        return _FirstToken.apply(h)
    return h[:, 0].contiguous()


class _EmbeddingResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pos_w, tok_w, S):
        H = pos_w.shape[1]
        r = torch.empty(1, S, H, dtype=pos_w.dtype, device=pos_w.device)
        call("ddl_rows_add_row", dcode(r), p(r), p(pos_w), p(tok_w), S, H)
        ctx.params = (pos_w, tok_w)
        ctx.S = S
        return r

    @staticmethod
    def backward(ctx, dr):
        pos_w, tok_w = ctx.params
        S, H = ctx.S, pos_w.shape[1]
        dr = dr.reshape(S, H).contiguous()
        if dr.dtype != pos_w.dtype:
            dr = dr.to(pos_w.dtype)
        sp, st = grad_sink(pos_w), grad_sink(tok_w)
        dpos = dtok = None
        if sp is not None:
            E.add_into(sp.view(-1)[:S * H], dr.view(-1))
            grad_ready(pos_w)
        else:
            dpos = torch.empty_like(pos_w)
            E.copy2d(dpos, dr, H, pos_w.shape[0], H, H, S, H)
        if st is not None:
            E.colsum(dr, st.view(-1)[:H], accumulate=True)
            grad_ready(tok_w)
        else:
            dtok = E.copy2d(torch.empty_like(tok_w), None, H, tok_w.shape[0], H)
            E.colsum(dr, dtok.view(-1)[:H])
        return dpos, dtok, None


def embedding_residual(pos_w: torch.Tensor, tok_w: torch.Tensor, S: int) -> torch.Tensor:
    """``pos_w[:S] + tok_w[0]`` as a [1, S, H] tensor."""
    H = pos_w.shape[1]
    if (pos_w.dtype == tok_w.dtype and pos_w.dtype in (torch.bfloat16, torch.float32) and S <= pos_w.shape[0]
            and H % 8 == 0 and _lib.use_native(pos_w, tok_w)):
        return _EmbeddingResidual.apply(pos_w, tok_w, S)
    return pos_w[:S].unsqueeze(0) + tok_w[0].view(1, 1, -1)


class _PrependTokenAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, head, table):
        B, P, H = x.shape
        S = P + 1
        x = x.contiguous()
        out = torch.empty(B, S, H, dtype=x.dtype, device=x.device)
        call("ddl_seq_prepend_add", dcode(x), p(out), p(x), p(head), p(table), B, S, H)
        ctx.params = (head, table)
        ctx.shape = (B, S, H)
        return out

    @staticmethod
    def backward(ctx, dout):
        head, table = ctx.params
        B, S, H = ctx.shape
        dout = dout.contiguous()
        d2 = dout.view(B, S * H)
        # patch tokens: rows 1.. of every sequence, one strided copy
        dx = torch.empty(B, S - 1, H, dtype=dout.dtype, device=dout.device)
        E.copy2d(dx.view(B, (S - 1) * H), d2[:, H:], (S - 1) * H, B, (S - 1) * H, S * H, B, (S - 1) * H)
        # position table: the column sums over the batch; the class token: their first row
        dtab = torch.empty(S * H, dtype=table.dtype, device=dout.device)
        E.colsum(d2, dtab)
        st, sh = grad_sink(table), grad_sink(head)
        dt = dh = None
        if st is not None:
            E.add_into(st.view(-1)[:S * H], dtab)
            grad_ready(table)
        else:
            dt = dtab.view(table.shape)
        if sh is not None:
            E.add_into(sh.view(-1)[:H], dtab[:H])
            grad_ready(head)
        else:
            dh = dtab[:H].clone().view(head.shape)
        return dx, dh, dt


def prepend_token_add(x: torch.Tensor, head: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    """``cat([head.expand(B, 1, H), x], 1) + table`` for x [B, P, H], head [1, 1, H] (or [H]), table
    [1, P + 1, H] (or [P + 1, H]) -- ViT's class token and position embeddings."""
    B, P, H = x.shape
    if (x.dtype == head.dtype == table.dtype and x.dtype in (torch.bfloat16, torch.float32)
            and head.numel() == H and table.numel() == (P + 1) * H and (P + 1) * H % 8 == 0
            and head.is_contiguous() and table.is_contiguous() and _lib.use_native(x, head, table)):
        return _PrependTokenAdd.apply(x, head, table)
    return torch.cat([head.reshape(1, 1, H).expand(B, -1, -1), x], 1) + table.reshape(1, P + 1, H)
