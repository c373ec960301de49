"""Looped nnet3 plan (host-only): context, chunk periodicity, priming, FLOPs."""
import pytest

from vosk import engine as ve


@pytest.mark.parametrize("fpc,priming", [(51, 1), (21, 3), (3, 17), (20, 3)])
def test_plan_context_and_priming(synth_model, fpc, priming):
    p = ve.plan_info(synth_model, fpc)
    assert p["fpc"] % 3 == 0 and p["fpc"] >= fpc
    # recipe topology: delta (+-2) + tdnnf2-4 (3x stride 1) + tdnnf6-12 (7x stride 3) = 26
    assert p["left_context"] == 26 and p["right_context"] == 26
    assert p["priming"] == priming
    assert p["out_dim"] == 2000


def test_plan_flops_match_recipe(synth_model):
    p = ve.plan_info(synth_model, 51)
    per_frame = p["flops_per_chunk"] / 17
    # ~7.9 MFLOP per output frame for the recipe topology
    assert 7.0e6 < per_frame < 8.5e6


def test_plan_fuses_component_chains(synth_model):
    d = ve.plan_describe(synth_model, 51)
    ops = [ln for ln in d.splitlines() if ln.strip().startswith(("GEMM", "GATHER"))]
    # one GEMM per affine-like component + the delta and input2 (delta + the
    # chunk's i-vector) gathers; the xent branch is pruned
    assert len(ops) == 30
    assert sum(1 for o in ops if "GATHER" in o) == 2
    assert not any("xent" in o for o in ops)
    assert any("-> LLH" in o for o in ops)
    # bias + relu + batchnorm + bypass fused into each TDNN-F affine
    assert sum(1 for o in ops if o.endswith("epi=0123")) == 11
