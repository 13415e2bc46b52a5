"""Pin the CPU oracle against fixtures produced by the reference itself (CPU only)."""
import numpy as np
import pytest

from golden_util import case_names, load_case, oracle_for, rel_nmse
from oracle.informer_np import AttnTrace, sample_shapes
from oracle.metrics_np import nmse_split

CASES = case_names()


def test_fixtures_present():
    assert {"informer_prob_b1", "informer_prob_b4", "transformer_c3", "informer_lsq8"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    case = load_case(name)
    orc = oracle_for(case)
    acts = {}
    if case.meta["model"] == "transformer":
        out = orc.forward(case.z["x_enc"], case.z["x_dec"], acts=acts)
        trace = None
    else:
        trace = AttnTrace()
        shapes = sample_shapes(orc.cfg)
        assert [tuple(s[1]) for s in shapes] == [i.shape for i in case.idx]
        out, attns = orc.forward(case.z["x_enc"], case.z["x_dec"], case.idx, acts=acts, trace=trace)
    ref = case.z["out"]
    assert out.shape == ref.shape
    assert rel_nmse(out, ref) < 1e-10, rel_nmse(out, ref)
    np.testing.assert_allclose(out, ref, rtol=2e-4, atol=2e-5)
    # per-stage activations recorded by reference forward hooks
    for k, v in case.acts().items():
        assert k in acts, k
        assert rel_nmse(acts[k], v) < 1e-10, (k, rel_nmse(acts[k], v))
    if trace is not None:
        n = case.meta["n_mtop"]
        assert len(trace.m_top) == n
        for k in range(n):
            np.testing.assert_array_equal(trace.m_top[k], case.z[f"mtop{k}"])
        if case.meta["model"] == "informer":     # Informer returns one encoder's per-layer maps
            attns = [attns]
        for key, a in case.z.items():
            if key.startswith("attn_e"):
                e, l = key[6:].split("_l")
                np.testing.assert_allclose(attns[int(e)][int(l)][0], a, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(nmse_split(ref, case.z["label"]), case.z["nmse_split"], rtol=1e-5)


def test_index_draws_are_torch_randint():
    """The recorded draws are mt19937 ``% L_K`` (see the engine's native sampler)."""
    from channelestimationtransformer_amd.rng import draw_indices

    for name in ("informer_prob_b1", "informer_prob_e43", "informer_prob_lab20"):
        case = load_case(name)
        # every ProbSparse call is a self-attention: L_K == L_Q
        shapes = [(i.shape[0], i.shape) for i in case.idx]
        got = draw_indices(shapes, seed=case.meta["rng_seed"])
        for g, i in zip(got, case.idx):
            np.testing.assert_array_equal(g, i)


@pytest.mark.parametrize("name", [n for n in CASES if n.startswith("informer")])
def test_torch_restatement_matches_reference(name):
    """oracle/informer_torch.py (the CPU baseline's forward: the reference's own aten ops) in float64
    against the reference fixtures."""
    import torch

    from golden_util import informer_oracle_config
    from oracle.informer_torch import TorchInformer

    case = load_case(name)
    bits = case.cfg.get("num_bits") if case.meta["model"] == "informer_lsq" else None
    cfg = informer_oracle_config(case.cfg, bits, stack=case.meta["model"] != "informer")
    m = TorchInformer(cfg, case.state, dtype=torch.float64)
    out = m.forward(torch.from_numpy(case.z["x_enc"]).double(), torch.from_numpy(case.z["x_dec"]).double(),
                    case.idx).numpy()
    assert rel_nmse(out, case.z["out"]) < 1e-10, rel_nmse(out, case.z["out"])


def test_host_cpu_description():
    from oracle.informer_torch import host_cpu

    h = host_cpu()
    assert h["usable_logical"] >= 1 and isinstance(h["model"], str)
