"""GPU parity of the layer-wise engine (shapes outside the fused kernels) against the reference.

The fixtures (tests/golden/make_golden.py) are the reference's own forwards at the shapes the
TimingAnalysis sweeps and the MimoSimulation checkpoint use: d_model 64 with e_layers [4,3];
5 heads of d_keys 25 (d_model // n_heads, attn.py:180-183) with d_ff 256; d_model 256 with 3 heads,
seq_len 48 and a genuinely sparse 34-row decoder; attn="full" at d_model 512.  The layer-wise
engine computes every contraction with fp32 operands on the f32 MFMA, so the bar is fp32-level:
rel-NMSE ≤ 1e-8 (measured ≈1e-12) — far inside the north star's 1e-4 — and the ProbSparse top-u
selection equals the reference's.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import case_names, layerwise_name, load_case, oracle_for, rel_nmse

pytestmark = pytest.mark.gpu

TOL = 1e-8
CASES = [n for n in case_names() if layerwise_name(n)]


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", CASES)
def test_layerwise_matches_reference_fixture(name):
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(name)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    assert eng.precision() == "fp32-layerwise"
    out, _, att = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, attns=bool(case.cfg["distil"]))
    assert np.isfinite(out).all()
    err = rel_nmse(out, case.z["out"])
    assert err < TOL, err
    # encoder attention maps of sequence 0 (output_attention <- distil in the callers' positional call)
    buf, layout, per = att
    k = 0
    for e, n in enumerate(case.cfg["e_layers"]):
        for l in range(n):
            key = f"attn_e{e}_l{l}"
            off, L = layout[k]
            k += 1
            if key not in case.z:
                continue
            a = buf[off:off + case.cfg["n_heads"] * L * L].reshape(case.cfg["n_heads"], L, L)
            assert rel_nmse(a, case.z[key]) < TOL, (key, rel_nmse(a, case.z[key]))


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("B", [1, 37])
def test_layerwise_random_batches_vs_oracle(name, B):
    """Batches of random sequences (every sequence its own): engine vs the float64 oracle."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(name)
    m = model_for(case)
    cfg = case.cfg
    rng = np.random.default_rng(B)
    xe = rng.standard_normal((B, cfg["seq_len"], cfg["enc_in"])).astype(np.float32)
    xd = rng.standard_normal((B, cfg["label_len"] + cfg["pred_len"], cfg["dec_in"])).astype(np.float32)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    ref, _ = oracle_for(case).forward(xe, xd, case.idx)
    assert rel_nmse(out, ref) < TOL


def test_layerwise_native_sampler_is_the_torch_stream():
    """cet_seed's host mirror of torch's mt19937 feeds the layer-wise path: a seeded forward equals the
    forward with the explicit torch.randint draws of the same seed."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_h5_ff256")
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    eng.seed(1)
    dev = torch.device("cuda:0")
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    out = torch.empty(xe.shape[0], case.cfg["pred_len"], 16, device=dev)
    eng.forward(xe, xd, out)
    torch.cuda.synchronize()
    assert rel_nmse(out.cpu().numpy(), case.z["out"]) < TOL   # the fixture's draws are torch.manual_seed(1)


def test_layerwise_route_for_a_fused_shape():
    """CET_LAYERWISE=1 routes even the C2 model through the layer-wise engine: it must agree with the
    reference fixture at fp32 level (a cross-check of the two engines' shared host plumbing)."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    os.environ["CET_LAYERWISE"] = "1"
    try:
        m = model_for(case)
        eng = m.engine(torch.device("cuda:0"))
    finally:
        del os.environ["CET_LAYERWISE"]
    assert eng.precision() == "fp32-layerwise"
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert rel_nmse(out, case.z["out"]) < TOL


def test_layerwise_nmse_split():
    """cet_forward_nmse on the layer-wise path: the standalone NMSE_Split after the forward."""
    _gpu()
    from engine_util import model_for

    from oracle.metrics_np import nmse_split

    case = load_case("informer_d64_e43")
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    eng.set_indices(case.idx)
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    lab = torch.from_numpy(case.z["label"]).to(dev)
    out = torch.empty(xe.shape[0], case.cfg["pred_len"], 16, device=dev)
    acc = torch.zeros(case.cfg["pred_len"], device=dev)
    eng.forward_nmse(xe, xd, out, lab, acc)
    torch.cuda.synchronize()
    np.testing.assert_allclose(acc.cpu().numpy(), nmse_split(out.cpu().numpy(), case.z["label"]), rtol=1e-5)
    np.testing.assert_allclose(acc.cpu().numpy(), case.z["nmse_split"], rtol=1e-4)


def test_layerwise_serving_loop_graph_over_caller_buffers():
    """A caller that repeats its buffers gets the operator sequence captured over them (no staging
    copies, cet_lw_host.cpp Model::forward): the repeated forwards, a forward on other buffers and a
    return to the first buffers all give the staged path's result bit for bit; the
    reference fixture's d_model-64 model (fused residual + LayerNorm epilogues)."""
    _gpu()
    from engine_util import model_for

    case = load_case("informer_d64_e43")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    rng = np.random.default_rng(11)
    B = 19
    xe_np = rng.standard_normal((B,) + case.z["x_enc"].shape[1:]).astype(np.float32)
    xd_np = rng.standard_normal((B,) + case.z["x_dec"].shape[1:]).astype(np.float32)
    xe, xd = torch.from_numpy(xe_np).to(dev), torch.from_numpy(xd_np).to(dev)
    def fwd(a, b, o):
        eng.set_indices(case.idx)   # the same ProbSparse draws every time (explicit indices last one forward)
        eng.forward(a, b, o)

    outs = []
    for _ in range(4):   # 1st: staged path, 2nd: capture over these buffers, 3rd/4th: that graph
        o = torch.empty(B, 5, 16, device=dev)
        fwd(xe, xd, o)
        outs.append(o)
    o_same = torch.empty(B, 5, 16, device=dev)
    for _ in range(3):
        fwd(xe, xd, o_same)
    xe2, xd2 = xe.clone(), xd.clone()
    o2 = torch.empty(B, 5, 16, device=dev)
    fwd(xe2, xd2, o2)
    fwd(xe, xd, o_same)
    torch.cuda.synchronize()
    ref = outs[0].cpu().numpy()
    for o in outs[1:] + [o_same, o2]:
        np.testing.assert_array_equal(o.cpu().numpy(), ref)
    orc, _ = oracle_for(case).forward(xe_np, xd_np, case.idx)
    assert rel_nmse(ref, orc) < TOL



CKPT = "informer_d64_s25_full"   # the MimoSimulation checkpoint architecture (Predict.py:91-93)


def _random_batch(cfg, B, seed):
    rng = np.random.default_rng(seed)
    xe = rng.standard_normal((B, cfg["seq_len"], cfg["enc_in"])).astype(np.float32)
    xd = rng.standard_normal((B, cfg["label_len"] + cfg["pred_len"], cfg["dec_in"])).astype(np.float32)
    return xe, xd


@pytest.mark.parametrize("B", [37, 512])
def test_fused_layerwise_checkpoint_fixture_and_oracle(B):
    """The checkpoint architecture (d_model 64, seq_len 25, e_layers [4,3], attn "full") runs on the fused
    layer-wise form (one workgroup per sequence, every activation in LDS): the fixture's inputs against
    the reference's own output, a random batch against the float64 oracle (a 64-row slice), and a
    repeated forward bit for bit."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(CKPT)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert eng.last_path() == "layerwise-fused"
    assert rel_nmse(out, case.z["out"]) < TOL, rel_nmse(out, case.z["out"])
    xe, xd = _random_batch(case.cfg, B, 100 + B)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    again, _, _ = run_engine(m, xe, xd, case.idx)
    assert eng.last_path() == "layerwise-fused"
    np.testing.assert_array_equal(out, again)
    n = min(B, 64)
    ref, _ = oracle_for(case).forward(xe[:n], xd[:n], case.idx)
    assert rel_nmse(out[:n], ref) < TOL, rel_nmse(out[:n], ref)


def test_fused_layerwise_equals_operator_launches():
    """The fused form and the operator-launch form of one model agree at fp32 rounding level (same
    arithmetic class; the softmax and P·V sums run in another order); a forward that materialises the
    attention maps keeps the operator launches."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(CKPT)
    xe, xd = _random_batch(case.cfg, 96, 5)
    m = model_for(case)
    fused, _, _ = run_engine(m, xe, xd, case.idx)
    assert m.engine(torch.device("cuda:0")).last_path() == "layerwise-fused"
    os.environ["CET_LW_FUSED"] = "0"   # read when the engine uploads its weights (first forward)
    try:
        m2 = model_for(case)
        eng2 = m2.engine(torch.device("cuda:0"))
        ops, _, _ = run_engine(m2, xe, xd, case.idx)
    finally:
        del os.environ["CET_LW_FUSED"]
    assert eng2.last_path() == "layerwise"
    assert rel_nmse(fused, ops) < 1e-11, rel_nmse(fused, ops)
    run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, attns=True)
    assert m.engine(torch.device("cuda:0")).last_path() == "layerwise"


@pytest.mark.parametrize("B", [3, 256])
def test_fused_layerwise_probsparse_vs_oracle(B):
    """The same architecture with attn "prob" (attn.py:73-175): the first encoder layer is genuinely
    sparse (u = 5·ceil(ln 25) = 20 of 25 queries: rank top-u, mean(V) rows), the decoder self-attention
    causal with mix; explicit draws, fused form against the float64 oracle at fp32 level."""
    _gpu()
    import dataclasses

    from engine_util import model_for, run_engine

    from channelestimationtransformer_amd.rng import draw_indices
    from oracle.informer_np import sample_shapes

    base = load_case(CKPT)
    meta = dict(base.meta)
    meta["cfg"] = dict(base.cfg, attn="prob")
    case = dataclasses.replace(base, meta=meta)
    orc = oracle_for(case)
    idx = draw_indices(sample_shapes(orc.cfg), seed=9)
    m = model_for(case)
    xe, xd = _random_batch(case.cfg, B, 7 + B)
    out, _, _ = run_engine(m, xe, xd, idx)
    assert m.engine(torch.device("cuda:0")).last_path() == "layerwise-fused"
    n = min(B, 64)
    ref, _ = orc.forward(xe[:n], xd[:n], idx)
    assert rel_nmse(out[:n], ref) < TOL, rel_nmse(out[:n], ref)


@pytest.mark.parametrize("attn,seq_len,label_len,pred_len", [("full", 48, 10, 5), ("prob", 48, 25, 9)])
def test_fused_layerwise_longer_shapes_vs_oracle(attn, seq_len, label_len, pred_len):
    """The fused layer-wise form past the checkpoint's own shape, with the checkpoint's weights (they do
    not depend on the lengths): seq_len 48 makes three m-tiles per GEMM; attn "full" gives 48 selected
    rows (the one-lane-per-row softmax, nsel > 32); attn "prob" with label_len 25 + pred_len 9 gives a
    genuinely sparse masked decoder (u = 5·ceil(ln 34) = 20 of 34 queries: unselected rows take cumsum(V),
    with the mix re-view).  Explicit draws, fused form against the float64 oracle at fp32 level."""
    _gpu()
    import dataclasses

    from engine_util import model_for, run_engine

    from channelestimationtransformer_amd.rng import draw_indices
    from oracle.informer_np import sample_shapes

    base = load_case(CKPT)
    meta = dict(base.meta)
    meta["cfg"] = dict(base.cfg, attn=attn, seq_len=seq_len, label_len=label_len, pred_len=pred_len)
    case = dataclasses.replace(base, meta=meta)
    orc = oracle_for(case)
    idx = draw_indices(sample_shapes(orc.cfg), seed=11)
    m = model_for(case)
    B = 37
    xe, xd = _random_batch(case.cfg, B, 5)
    out, _, _ = run_engine(m, xe, xd, idx)
    assert m.engine(torch.device("cuda:0")).last_path() == "layerwise-fused"
    ref, _ = orc.forward(xe, xd, idx)
    assert rel_nmse(out, ref) < TOL, rel_nmse(out, ref)
    # the same forward on the operator launches agrees with the fused form
    os.environ["CET_LW_FUSED"] = "0"
    try:
        m2 = model_for(case)
        out2, _, _ = run_engine(m2, xe, xd, idx)
        assert m2.engine(torch.device("cuda:0")).last_path() == "layerwise"
    finally:
        del os.environ["CET_LW_FUSED"]
    assert rel_nmse(out, out2) < 1e-10, rel_nmse(out, out2)


@pytest.mark.parametrize("seq_len,path", [(32, "layerwise-fused"), (48, "layerwise")])
def test_fused_layerwise_stack_output_rows_bound(seq_len, path):
    """The fused layer-wise GEMM covers at most 3 m-tiles (48 rows), and the decoder's cross-attention K/V
    GEMM runs over S = the stack output's rows.  e_layers [1, 1] (no distil conv in a one-layer encoder,
    encoder.py:95-106) gives S = seq_len + seq_len/2: 48 at seq_len 32 (fused), 72 at seq_len 48, which
    must take the operator launches.  Seeded synthetic weights, d_model 64 (layer-wise shapes), attn
    "full", against the float64 oracle."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, seq_len, 10, 5, 5, 64, 4, [1, 1], 2, 64, 0.05, "full", "fixed", "gelu", False,
                      True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 4).items()})
    m.eval()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    orc = InformerOracle(InformerConfig(seq_len=seq_len, d_model=64, n_heads=4, e_layers=(1, 1), d_layers=2,
                                        attn="full"), state)
    B = 21
    xe, xd, _ = make_batch(B, seed=41)
    xe = np.ascontiguousarray(xe[:, -seq_len:])
    with torch.no_grad():
        res = m(torch.from_numpy(xe).to(dev), range(seq_len), torch.from_numpy(xd).to(dev), range(15))
    out = (res[0] if isinstance(res, tuple) else res).cpu().numpy()
    assert m.engine(dev).last_path() == path
    ref, _ = orc.forward(xe, xd, ())
    assert rel_nmse(out, ref) < TOL, rel_nmse(out, ref)


BF16_TOL = 1e-4   # the north star's tolerance (BASELINE.json) for bf16 operands


@pytest.mark.parametrize("B", [1, 512])
def test_fused_layerwise_bf16_checkpoint_vs_oracle(B):
    """bf16 GEMM operands in the fused layer-wise form (cet_set_precision "bf16" on a layer-wise engine; the
    compile-time d_model-64 instance, v_mfma_f32_16x16x32_bf16 with fp32 accumulation, LayerNorm and
    attention): the checkpoint fixture against the reference's own output and a random batch's row slices
    against the float64 oracle, both within the north star's 1e-4 — and above the fp32 bar, so the bf16
    instance is the one that ran —; a repeated forward bit for bit."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(CKPT)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    eng.set_precision("bf16")
    assert eng.precision() == "bf16"
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert eng.last_path() == "layerwise-fused"
    assert eng.last_kernel() == "cet::lw::lw_fused (bf16 operands)"
    err = rel_nmse(out, case.z["out"])
    assert TOL < err < BF16_TOL, err
    xe, xd = _random_batch(case.cfg, B, 300 + B)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    again, _, _ = run_engine(m, xe, xd, case.idx)
    np.testing.assert_array_equal(out, again)
    rows = np.r_[0:32, B - 32:B] if B > 64 else np.arange(B)
    ref, _ = oracle_for(case).forward(xe[rows], xd[rows], case.idx)
    err = rel_nmse(out[rows], ref)
    assert err < BF16_TOL, err


def test_fused_layerwise_bf16_runtime_shapes_and_refusals():
    """The bf16 operands on the runtime-shape instance (seq_len 48: three m-tiles per GEMM, 48 selected rows
    — the one-lane-per-row softmax —, a 34-row decoder) against the float64 oracle within 1e-4, attn "full":
    with a genuinely sparse ProbSparse call bf16 rounding of the scores can flip the top-u selection, an
    output discontinuity no operand precision short of fp32 bounds (measured 0.12 on a sparse causal decoder;
    the v4 kernel's "auto" takes split bf16 there).  A forward that materialises attention maps
    (operator launches only) is refused, not run in fp32; "auto" stays fp32."""
    _gpu()
    import dataclasses

    from engine_util import model_for, run_engine

    from channelestimationtransformer_amd.rng import draw_indices
    from oracle.informer_np import sample_shapes

    base = load_case(CKPT)
    meta = dict(base.meta)
    meta["cfg"] = dict(base.cfg, attn="full", seq_len=48, label_len=25, pred_len=9)
    case = dataclasses.replace(base, meta=meta)
    orc = oracle_for(case)
    idx = draw_indices(sample_shapes(orc.cfg), seed=13)
    assert not len(idx)   # attn "full": no draws
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    assert eng.precision() == "fp32-layerwise"
    eng.set_precision("bf16")
    xe, xd = _random_batch(case.cfg, 41, 17)
    out, _, _ = run_engine(m, xe, xd, idx)
    assert eng.last_path() == "layerwise-fused"
    assert eng.last_kernel() == "cet::lw::lw_fused (bf16 operands)"
    ref, _ = orc.forward(xe, xd, idx)
    err = rel_nmse(out, ref)
    assert TOL < err < BF16_TOL, err
    with pytest.raises(Exception, match="bf16 operands need the fused"):
        run_engine(m, xe, xd, idx, attns=True)
    with pytest.raises(Exception):
        eng.set_precision("split-bf16")


def test_fused_layerwise_bf16_deep_k_vs_oracle():
    """bf16 operands on the runtime-shape fused layer-wise instance with GEMMs deeper than 256: d_model 128
    with a distil conv (K = 3·128 = 384) and d_ff 320 (FFN2 K = 320).  The runtime-K bf16 loop runs every
    32-feature k-step of these (it once stopped after 8).  Seeded synthetic weights, attn "full"
    (no selection flips under bf16), against the float64 oracle within the north star's 1e-4 and above the
    fp32 bar, so the bf16 instance is what ran."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    dev = torch.device("cuda:0")
    seq_len = 32
    m = InformerStack(16, 16, 16, seq_len, 10, 5, 5, 128, 4, [2], 1, 320, 0.05, "full", "fixed", "gelu", False,
                      True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 6).items()})
    m.eval()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    orc = InformerOracle(InformerConfig(seq_len=seq_len, d_model=128, n_heads=4, e_layers=(2,), d_layers=1,
                                        d_ff=320, attn="full"), state)
    eng = m.engine(dev)
    eng.set_precision("bf16")
    B = 19
    xe, xd, _ = make_batch(B, seed=43)
    xe = np.ascontiguousarray(xe[:, -seq_len:])
    with torch.no_grad():
        res = m(torch.from_numpy(xe).to(dev), range(seq_len), torch.from_numpy(xd).to(dev), range(15))
    out = (res[0] if isinstance(res, tuple) else res).cpu().numpy()
    assert eng.last_path() == "layerwise-fused"
    assert eng.last_kernel() == "cet::lw::lw_fused (bf16 operands)"
    ref, _ = orc.forward(xe, xd, ())
    err = rel_nmse(out, ref)
    assert TOL < err < BF16_TOL, err
