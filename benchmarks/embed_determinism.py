"""Run-to-run bit equality of the word-embedding gradient: sorted segmented sum (default) vs the
fp32-atomic scatter (DDL_EMBED_SORTED=0 path), on a BERT-shaped batch with repeated ids
(a [CLS]-like id at position 0, padding id 0 over the last 38 positions)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from databricks_distributed_deep_learning_amd.ops import _native_embedding as Em  # noqa: E402


def main(reps: int = 8):
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    w = torch.randn(30522, 768, device=dev).bfloat16()
    ids = torch.randint(0, 30522, (128, 128), device=dev)
    ids[:, 0] = 101
    ids[:, 90:] = 0
    g = torch.randn(128, 128, 768, device=dev).bfloat16()
    for sorted_path in (True, False):
        Em._SORTED = sorted_path
        outs = []
        for _ in range(reps):
            ww = w.clone().requires_grad_(True)
            Em.embedding(ids, ww).backward(g)
            outs.append(ww.grad.clone())
        torch.cuda.synchronize()
        diff = [int((o != outs[0]).any(dim=1).sum().item()) for o in outs[1:]]
        print(f"{'sorted' if sorted_path else 'atomic'}: rows differing from run 0 in runs 1..{reps - 1}: {diff}")
    Em._SORTED = True


if __name__ == "__main__":
    main()
