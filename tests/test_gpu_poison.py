"""LDS poison: the v4 kernels' outputs do not depend on what a CU's LDS held before the workgroup started.

With CET_LDS_POISON=1 every v4 kernel (the fused Informer in every instance, the fused Transformer) fills its
whole dynamic LDS allocation with 0xFF bytes — NaN as fp32, bf16 and e4m3 — at entry, before it stages or
zeroes anything.  The entry code of cet_informer4.hpp zeroes only the image rows an MFMA can read before
anything writes them and argues that every other row below L is written by the first layer before any later
layer or the decoder reads it.  A read the argument misses would take whatever the CU's previous workgroup
left (finite garbage passes a tolerance, NaN garbage poisons a sequence: the round-5 r05c failure class);
under the poison it is a deterministic NaN.  So each case runs twice, poisoned and not, and the two outputs
must be bitwise equal, finite and within the north star's 1e-4 of the reference (the reference's own fixture
output, or the float64 oracle on row slices).  Reference: attn.py:116-146 (the rows the attention reads),
encoder.py:6-106, decoder.py:28-56.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import case_names, layerwise_name, load_case, oracle_for, rel_nmse

pytestmark = pytest.mark.gpu

TOL = 1e-4
INFORMER_CASES = [n for n in case_names() if n.startswith("informer") and not layerwise_name(n)]


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _twice(run):
    """run() without and with the poison; returns (plain, poisoned)."""
    plain = run()
    os.environ["CET_LDS_POISON"] = "1"
    try:
        poisoned = run()
    finally:
        del os.environ["CET_LDS_POISON"]
    return plain, poisoned


@pytest.mark.parametrize("instance", ["production", "diag"])
@pytest.mark.parametrize("name", INFORMER_CASES + ["transformer_c3"])
def test_fixture_under_lds_poison(name, instance):
    """Every v4 reference fixture (both Informer instances, and the Transformer) poisoned vs not: bitwise
    equal, and within 1e-4 of the reference's own output."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(name)
    m = model_for(case)
    diag = instance == "diag"

    def run():
        out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=diag)
        return out

    plain, poisoned = _twice(run)
    assert np.isfinite(poisoned).all()
    np.testing.assert_array_equal(poisoned, plain)
    err = rel_nmse(poisoned, case.z["out"])
    assert err < TOL, err


@pytest.mark.parametrize("e_layers,B", [([4, 3], 64), ([4, 3], 1), ([3, 2, 1], 5), ([3, 2, 1], 170)])
def test_encoder_split_under_lds_poison(e_layers, B):
    """The encoder split (one workgroup per encoder of a sequence; the last arrival fetches the other
    encoders' rows and runs the decoder, and zeroes only its own window's rows at entry) poisoned vs not:
    bitwise equal, and against the float64 oracle."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, e_layers, 3, 64, 0.05, "full", "fixed", "gelu", False,
                      True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 5).items()})
    m.eval()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    xe, xd, _ = make_batch(B, seed=310 + B)

    def run():
        with torch.no_grad():
            res = m(torch.from_numpy(xe).to(dev), range(90), torch.from_numpy(xd).to(dev), range(15))
        return (res[0] if isinstance(res, tuple) else res).cpu().numpy()

    plain, poisoned = _twice(run)
    assert m.engine(dev).last_path() == "v4-split"
    assert np.isfinite(poisoned).all()
    np.testing.assert_array_equal(poisoned, plain)
    rows = np.arange(B) if B <= 16 else np.r_[0:8, B - 8:B]
    ref, _ = InformerOracle(InformerConfig(e_layers=tuple(e_layers), attn="full"), state).forward(xe[rows], xd[rows], ())
    assert rel_nmse(poisoned[rows], ref) < TOL


@pytest.mark.parametrize("attn", ["prob", "full"])
def test_c2_instance_b512_under_lds_poison(attn):
    """The benchmarked C2 instance at B = 512 (every CU holds two workgroups) with the fused NMSE_Split,
    poisoned vs not: outputs and NMSE sums bitwise equal, and row slices against the float64 oracle."""
    _gpu()
    from engine_util import model_for

    from channelestimationtransformer_amd.dataset import make_batch

    case = load_case("informer_prob_b4")
    import dataclasses
    meta = dict(case.meta)
    meta["cfg"] = dict(case.cfg, attn=attn)
    case = dataclasses.replace(case, meta=meta)
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    B = 512
    xe_np, xd_np, lab_np = make_batch(B, seed=2024)
    xe = torch.from_numpy(xe_np).to(dev)
    xd = torch.from_numpy(xd_np).to(dev)
    lab = torch.from_numpy(np.ascontiguousarray(lab_np, np.float32)).to(dev)
    idx = case.idx if attn == "prob" else ()

    def run():
        out = torch.empty(B, 5, 16, device=dev)
        acc = torch.zeros(5, device=dev)
        sums = torch.zeros(10, dtype=torch.float64, device=dev)
        if len(idx):
            eng.set_indices(idx)
        eng.forward_nmse(xe, xd, out, lab, acc, sums)
        torch.cuda.synchronize()
        return out.cpu().numpy(), sums.cpu().numpy()

    (p_out, p_sums), (q_out, q_sums) = _twice(run)
    assert eng.last_kernel() == "cet::v4::informer_forward_v4<64, false, 0, false, 1, false, false, 0>"
    assert np.isfinite(q_out).all()
    np.testing.assert_array_equal(q_out, p_out)
    np.testing.assert_array_equal(q_sums, p_sums)
    rows = np.r_[0:16, B - 16:B]
    ref, _ = oracle_for(case).forward(xe_np[rows], xd_np[rows], idx)
    assert rel_nmse(q_out[rows], ref) < TOL
