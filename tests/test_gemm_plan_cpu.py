"""GEMM tuner candidate lists (ops/_native_gemm.py): pure host logic, no GPU.

* the "hybrid" row split is offered exactly when a 256x256-tile grid ends in a partial round and
  the remainder can be split-K over the chip (ViT-B/16: 297 / 891 tiles; not BERT-base's 192 /
  768-tile grids, which are under one round or whole rounds);
* its first launch covers whole rounds of tiles, so the split part is the partial round only;
* "big192" (256 x 192 tiles) is opt-in (DDL_GEMM_192=1) and only for N % 192 == 0.
"""
import importlib

import pytest

NG = importlib.import_module("databricks_distributed_deep_learning_amd.ops._native_gemm")


@pytest.mark.parametrize("M,N,K,expect", [
    (25216, 768, 768, (21760, 3)),      # ViT O-projection: 99 x 3 = 297 tiles
    (25216, 768, 3072, (21760, 6)),     # ViT FFN2: same grid, K = 3072 allows 6 splits
    (25216, 2304, 768, (21760, 2)),     # ViT QKV: 99 x 9 = 891 tiles, 126-tile remainder
    (16384, 768, 768, None),            # BERT: 192 tiles, under one round
    (16384, 3072, 768, None),           # BERT FFN1: 768 tiles, three whole rounds
    (25216, 3072, 768, None),           # ViT FFN1: 168-tile remainder cannot split within one round
    (25216, 768, 200, None),            # K not a whole number of 64-wide k-tiles
])
def test_hybrid_rows(M, N, K, expect):
    assert NG.hybrid_rows(M, N, K) == expect
    if expect is not None:
        m1, s = expect
        tn = -(-N // 256)
        assert m1 % 256 == 0 and (m1 // 256) * tn <= ((-(-M // 256) * tn) // NG.NUM_CU) * NG.NUM_CU
        assert (-(-(M - m1) // 256)) * tn * s <= NG.NUM_CU


def test_candidates_offer_hybrid_only_for_partial_rounds():
    kinds = {c[0] for c in NG._candidates(NG.MODE_NT, 25216, 768, 3072, False, 3072, 3072)}
    assert "hybrid" in kinds and "big" in kinds
    kinds = {c[0] for c in NG._candidates(NG.MODE_NT, 16384, 768, 3072, False, 3072, 3072)}
    assert "hybrid" not in kinds
    # weight-gradient (TN) and row-remapped GEMMs never take it
    assert not any(c[0] == "hybrid" for c in NG._candidates(NG.MODE_TN, 25216, 768, 3072, False, 768, 3072))
    assert not any(c[0] == "hybrid" for c in NG._candidates(NG.MODE_NT, 25216, 768, 3072, True, 3072, 3072))


def test_big192_candidate(monkeypatch):
    """256 x 192 tiles are offered for N % 192 == 0 NT / NN GEMMs (DDL_GEMM_192=0 drops them)."""
    monkeypatch.setattr(NG, "_BIG192", False)
    assert not any(c[0] == "big192" for c in NG._candidates(NG.MODE_NT, 16384, 768, 768, False, 768, 768))
    monkeypatch.setattr(NG, "_BIG192", True)
    assert ("big192", 1) in NG._candidates(NG.MODE_NT, 16384, 768, 768, False, 768, 768)
    assert ("big192", 1) in NG._candidates(NG.MODE_NN, 16384, 2304, 768, False, 768, 2304)
    assert not any(c[0] == "big192" for c in NG._candidates(NG.MODE_NT, 16384, 1024, 768, False, 768, 768))


def test_no_vendor_gemm_kind():
    """Every tuner candidate is a kernel of this library: a stale plan entry naming another
    kind (e.g. the removed hipBLASLt "blas" candidate) falls back to the native heuristic."""
    assert "blas" not in NG._KINDS and not hasattr(NG, "_blas")
    for mode in (NG.MODE_NT, NG.MODE_NN, NG.MODE_TN):
        assert all(k in NG._KINDS for k, _ in NG._candidates(mode, 16384, 768, 768, False, 768, 768, plain=True))


def test_online_tuning_commits_in_model_argmin(monkeypatch):
    """In-model tuning: calls of an untuned signature cycle through its candidates while the
    session is open; the committed choice is the candidate with the lowest median sample."""
    import contextlib

    class Ev:
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

        def synchronize(self):
            pass

    monkeypatch.setattr(NG, "_TUNE", True)
    monkeypatch.setattr(NG, "_ONLINE", True)
    monkeypatch.setattr(NG.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(NG.torch.cuda, "synchronize", lambda *a: None)
    NG._online.clear()
    key = "k-online"
    cands = [("big", 1), ("small", 2), ("big192", 1)]
    times = {("big", 1): [5.0, 5.2, 4.9], ("small", 2): [6.0, 3.0, 6.5], ("big192", 1): [4.0, 4.1, 9.0]}
    with NG.online_tuning(True):
        assert NG._online_active
        st = NG._online[key] = {"cands": cands, "n": 0, "pending": [], "samples": {}}
        for i in range(9):
            c = st["cands"][st["n"] % 3]
            st["n"] += 1
            t = times[c][i // 3]
            st["pending"].append((c, Ev(0.0), Ev(t)))
        NG.online_collect()
        assert st["samples"][("small", 2)] == [6.0, 3.0, 6.5] and not st["pending"]
    assert not NG._online_active and key not in NG._online
    assert NG._tuned.pop(key) == ("big192", 1)          # medians 5.0 / 6.0 / 4.1
    assert NG._timings.pop(key)[("small", 2)] == 6.0


def test_online_tuning_default_and_byte_gate(monkeypatch):
    """DDL_GEMM_TUNE_ONLINE unset: the caller's default decides (the trainer passes True for
    transformer models); "0" / "1" override it; max_mb keeps signatures over the gate on the
    isolated tuner and is restored on exit."""
    monkeypatch.setattr(NG, "_TUNE", True)
    monkeypatch.setattr(NG.torch.cuda, "is_available", lambda: True)
    for env, default, want in ((None, True, True), (None, False, False), ("0", True, False), ("1", False, True)):
        monkeypatch.setattr(NG, "_ONLINE_ENV", env)
        monkeypatch.setattr(NG, "_ONLINE", env == "1")
        with NG.online_tuning(True, default=default, max_mb=64):
            assert NG._online_active == want, (env, default)
            assert NG._online_max_bytes == 64 * 2 ** 20
        assert not NG._online_active and NG._online_max_bytes == float("inf")
    # the trainer's rule: transformers tune in-model with no gate, CNNs stay on the isolated tuner
    from databricks_distributed_deep_learning_amd.config import get_preset
    for preset, online in (("bert_base_ddp", True), ("vit_b16", True), ("resnet50_ddp", False)):
        m = get_preset(preset).model
        assert m.startswith(("bert", "vit", "gpt", "t5", "roberta")) == online, m


def test_wg_candidate(monkeypatch):
    """The 4-wave weight-gradient kernel is offered for plain TN GEMMs inside its contract
    (M % 256, N % 128, K % 128) -- BERT-base's four weight gradients -- and nowhere else."""
    monkeypatch.setattr(NG, "_WG", True)
    for M, N in [(2304, 768), (768, 3072), (3072, 768), (768, 768)]:
        c = NG._candidates(NG.MODE_TN, M, N, 16384, False, M, N, plain=True)
        assert any(k == "wg" for k, _ in c), (M, N)
        assert all(s >= 1 for k, s in c if k == "wg")
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_TN, 200, 256, 16384, False, 200, 256, plain=True))
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_TN, 256, 256, 16400, False, 256, 256, plain=True))
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_TN, 768, 768, 16384, False, 768, 768, plain=False))
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_NT, 768, 768, 16384, False, 768, 768, plain=True))
    monkeypatch.setattr(NG, "_WG", False)
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_TN, 768, 768, 16384, False, 768, 768, plain=True))


def test_wg_candidate_conv_wgrad(monkeypatch):
    """Conv weight gradients (CONVW) get the 4-wave kernel when the input channel count keeps each
    8-channel chunk inside one tap (C % 8 == 0) and the GEMM is inside its contract."""
    monkeypatch.setattr(NG, "_WG", True)
    c = NG._candidates(NG.MODE_CONVW, 256, 2304, 50176, False, 256, 0, plain=True, conv_c=256)
    assert any(k == "wg" for k, _ in c)
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_CONVW, 256, 2304, 50176, False, 256, 0, plain=True))
    assert not any(k == "wg" for k, _ in NG._candidates(NG.MODE_CONVW, 256, 1152, 50176, False, 256, 0, plain=True,
                                                         conv_c=4))


def test_duo_candidate_contract():
    """The dual-workgroup kernel ("duo", gemm_duo.hip) is a tuner candidate for NT / NN GEMMs with
    N % 128 == 0, K % 32 == 0 and the epilogues it implements -- never for TN, convolutions, fp32
    outputs, accumulation or a GELU with a residual."""
    import torch
    b = torch.zeros(768, dtype=torch.bfloat16)
    ok = NG.duo_ok
    assert ok(NG.MODE_NT, 16384, 3072, 768, 768, 768, 3072, b, "gelu", object(), None, None)
    assert ok(NG.MODE_NN, 16384, 3072, 768, 768, 3072, 3072, None, "dgelu", object(), None, object())
    assert ok(NG.MODE_NN, 25216, 768, 3072, 3072, 768, 768, None, None, None, object(), None)
    assert not ok(NG.MODE_TN, 768, 768, 16384, 768, 768, 768, None, None, None, None, None)
    assert not ok(NG.MODE_NT, 16384, 1000, 768, 768, 768, 1000, None, None, None, None, None)
    assert not ok(NG.MODE_NT, 16384, 768, 200, 200, 200, 768, None, None, None, None, None)
    assert not ok(NG.MODE_NT, 16384, 3072, 768, 768, 768, 3072, b, "gelu", object(), object(), None)
    assert not ok(NG.MODE_NT, 16384, 3072, 768, 768, 768, 3072, b.float(), None, None, None, None)
    assert not ok(NG.MODE_NN, 16384, 768, 768, 768, 768, 768, None, None, None, None, None, accumulate=True)
    assert not ok(NG.MODE_NT, 16384, 768, 768, 768, 768, 768, None, "relu", None, None, None)
    cands = NG._tune_candidates(NG.MODE_NT, 16384, 3072, 768, 768, 768, b, "gelu", object(), False, None, None)
    assert ("duo", 1) in cands
    cands = NG._tune_candidates(NG.MODE_TN, 768, 3072, 16384, 768, 3072, None, None, None, False, None, None)
    assert ("duo", 1) not in cands


# ---------------------------------------------------------------- committed plan table
def _fresh_table(monkeypatch, tmp_path, doc, arch="gfx950", src="abc"):
    path = tmp_path / "plans.json"
    path.write_text(__import__("json").dumps(doc))
    monkeypatch.setattr(NG, "_TABLE_ENV", str(path))
    monkeypatch.setattr(NG, "_TABLE_PATH", str(path))
    monkeypatch.setattr(NG, "_table", None)
    monkeypatch.setattr(NG, "_table_info", dict(NG._table_info))
    monkeypatch.setattr(NG, "_device_arch", lambda: arch)
    monkeypatch.setattr(NG._lib, "gemm_src_hash", lambda: src)
    return NG.load_plan_table()


def test_plan_table_loads_for_matching_arch_and_sources(monkeypatch, tmp_path):
    """The committed table applies only to the GPU architecture and GEMM-kernel build it was tuned
    on: another source hash or architecture leaves it unused (tuning takes over)."""
    doc = {"gfx950": {"gemm_src_hash": "abc", "plans": {"0|16384|768|768": ["big192", 1], "2|768|768|16384": ["duo", 4]}}}
    t = _fresh_table(monkeypatch, tmp_path, doc)
    assert t == {"0|16384|768|768": ("big192", 1), "2|768|768|16384": ("duo", 4)}
    assert NG.plan_stats()["status"] == "loaded" and NG.plan_stats()["entries"] == 2
    assert _fresh_table(monkeypatch, tmp_path, doc, src="other") == {}
    assert NG.plan_stats()["status"].startswith("stale")
    assert _fresh_table(monkeypatch, tmp_path, doc, arch="gfx942") == {}
    assert _fresh_table(monkeypatch, tmp_path, doc, src=None) == {}


def test_plan_table_is_in_sync_with_the_tree():
    """ops/gemm_plans.json's gfx950 entry was tuned against the GEMM kernel sources in this tree
    (a kernel edit without re-tuning would silently drop the committed plan: the bench's
    plan_source would read 'tuned').  Every entry names a kernel kind the launcher knows."""
    import json
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "csrc"))
    import build as native_build
    with open(os.path.join(root, "databricks_distributed_deep_learning_amd", "ops", "gemm_plans.json")) as f:
        doc = json.load(f)
    ent = doc["gfx950"]
    assert ent["gemm_src_hash"] == native_build.gemm_src_hash()
    assert len(ent["plans"]) > 50
    for k, (kind, s) in ent["plans"].items():
        if k.startswith("dgrad_path|"):       # strided-conv dgrad path (ops/_native_conv.py)
            assert kind in ("serial", "multi", "multi_narrow"), (k, kind)
        else:
            assert kind in NG._KINDS and int(s) >= 1, (k, kind, s)
