"""GPU parity of the fused InformerStack kernel against the reference fixtures and the oracle.

Tolerance: the north star's 1e-4 relative NMSE (Σ(a-b)²/Σb²) vs the reference fp32 CPU
forward.  The engine computes GEMM/attention operands in bf16 with fp32 accumulation,
LayerNorm/softmax/residual in fp32.
"""
import numpy as np
import pytest
import torch

from golden_util import case_names, layerwise_name, load_case, rel_nmse

pytestmark = pytest.mark.gpu

TOL = 1e-4
# the fused kernels' cases (the layer-wise engine's shapes: tests/test_gpu_layerwise.py)
INFORMER_CASES = [n for n in case_names() if n.startswith("informer") and not layerwise_name(n)]


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fixture_selection_mismatches(case, dbg):
    """(b, h) rows, summed over the sparse calls, where the engine's top-u (rebuilt from its dumped M with
    the same rank rule) differs from the reference's M_top recorded in the fixture."""
    n = 0
    for k in range(case.meta["n_mtop"]):
        Mk = dbg.get(f"M{k}")
        if Mk is None or not np.isfinite(Mk).all():      # u == L: every query selected
            continue
        mt = case.z[f"mtop{k}"]
        sel = np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :mt.shape[-1]], axis=-1)
        n += int((sel != mt).any(-1).sum())
    return n


@pytest.mark.parametrize("instance", ["production", "diag"])
@pytest.mark.parametrize("name", INFORMER_CASES)
def test_informer_matches_reference_fixture(name, instance):
    """Every reference fixture through both kernel instances: the production one (what bench.py and the
    configs tool time) and the diagnostic one (activation dumps; every dumped stage is checked against
    the oracle), at the engine's automatic precision.  A genuinely sparse masked decoder
    (informer_prob_lab20: L=25, u=20, unselected rows take cumsum(V)) is output-discontinuous in the
    top-u selection, so the engine runs it in split bf16 (v4) and its selection must equal the
    reference's M_top exactly."""
    _gpu()
    from engine_util import model_for, run_engine, stage_report

    case = load_case(name)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    diag = instance == "diag"
    out, dbg, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=diag)
    rep, _, _ = stage_report(case, out, dbg)
    err = rel_nmse(out, case.z["out"])
    assert np.isfinite(out).all()
    assert err < TOL, (err, rep)
    cfg = case.cfg
    Ld = cfg["label_len"] + cfg["pred_len"]
    sparse_dec = cfg["attn"] == "prob" and min(cfg["factor"] * int(np.ceil(np.log(Ld))), Ld) < Ld
    assert eng.precision() == ("split-bf16" if sparse_dec else "bf16")
    # which kernel ran: stacks without ProbSparse draws take the v4 encoder split at small batch (not with
    # the dumps), split bf16 runs on v4, the rest on the generation asked for
    split_ok = isinstance(cfg["e_layers"], (list, tuple)) and len(cfg["e_layers"]) > 1
    split_ok = split_ok and cfg["attn"] == "full" and case.meta["model"] != "informer" and not diag
    if sparse_dec:
        assert eng.last_path() == "v4"
    elif split_ok:
        assert eng.last_path() == "v4-split"
    else:
        assert eng.last_path() == "v4"
    if diag:   # every dumped stage (embedding, each layer, conv, encoder norms, decoder layers) vs the oracle
        bad = {k: v for k, v in rep.items() if not k.startswith("M") and not v < 1e-3}
        assert not bad, bad
    if diag and sparse_dec:
        assert fixture_selection_mismatches(case, dbg) == 0


SPLIT_TOL = 1e-8   # split bf16: ≈16 significant bits per operand, fp32 accumulation (measured ≤ 1e-10)


@pytest.mark.parametrize("name", INFORMER_CASES)
def test_split_bf16_is_fp32_parity(name):
    """Precision "split-bf16" on every fixture: fp32-level agreement with the reference and exactly
    the reference's top-u selection in every ProbSparse call (the M dumps of the DIAG instance), and
    the production instance bitwise equal to the DIAG instance."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(name)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    eng.set_precision("split-bf16")
    out, dbg, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=True)
    prod, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert rel_nmse(out, case.z["out"]) < SPLIT_TOL
    assert fixture_selection_mismatches(case, dbg) == 0
    np.testing.assert_array_equal(prod, out)


FP8_TOL = 2e-3   # e4m3 activations (3 mantissa bits: ≈3.6 % RMS rounding of every quantised GEMM input); measured 8.2e-4


def test_fp8_activations_lsq8():
    """C5 as BASELINE states it: LSQ 8-bit integer weights (exact, two e4m3 parts), fp8 e4m3
    activations on v_mfma_f32_16x16x32_fp8_fp8, fp32 accumulation / LayerNorm / softmax, against the
    reference's fp32 fake-quant forward; the production instance at B=1024 against the oracle."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from engine_util import model_for, run_engine
    from golden_util import oracle_for

    case = load_case("informer_lsq8")
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    eng.set_precision("fp8")
    assert eng.precision() == "fp8"
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert rel_nmse(out, case.z["out"]) < FP8_TOL
    xe, xd, _ = make_batch(1024, seed=77)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    rows = np.r_[0:32, 1024 - 32:1024]
    ref, _ = oracle_for(case).forward(xe[rows], xd[rows], case.idx)
    assert np.isfinite(out).all() and rel_nmse(out[rows], ref) < FP8_TOL


def test_fp8_refuses_non_lsq_and_wide_grids():
    _gpu()
    from engine_util import model_for

    for name in ("informer_prob_b4", "informer_lsq10"):
        m = model_for(load_case(name))
        eng = m.engine(torch.device("cuda:0"))
        eng.set_precision("fp8")
        with pytest.raises(Exception):
            eng.precision()


def test_lsq_grid_beyond_bf16_goes_split():
    """An LSQ grid with |q| > 256 (11 bits, steps 1/8 of the initialisation) is not exact in bf16: the
    automatic precision is split bf16, which carries it exactly; explicit bf16 is refused."""
    _gpu()
    from engine_util import model_for, run_engine
    from golden_util import oracle_for

    case = load_case("informer_lsq11")
    for k in list(case.state):
        if k.endswith("step_size"):
            case.state[k] = (np.asarray(case.state[k]) / 8).astype(np.float32)
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    assert eng.precision() == "split-bf16"
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    ref, _ = oracle_for(case).forward(case.z["x_enc"], case.z["x_dec"], case.idx)
    assert rel_nmse(out, ref) < SPLIT_TOL
    eng.set_precision("bf16")
    with pytest.raises(Exception):
        eng.precision()


def engine_selections(dbg, trace):
    """The engine's top-u per ProbSparse call, rebuilt from its dumped M (same rank rule)."""
    sels = []
    for k, mt in enumerate(trace.m_top):
        u = mt.shape[-1]
        Mk = dbg.get(f"M{k}")
        if Mk is None or not np.isfinite(Mk).all():   # u == L: every query selected
            sels.append(mt)
        else:
            sels.append(np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :u], axis=-1))
    return sels


@pytest.mark.parametrize("name", INFORMER_CASES)
def test_selection_conditional_parity_and_near_ties(name):
    """Given the engine's own top-u selection the forward matches the oracle to 1e-4, and every
    query where the selection differs from the oracle's is a near-tie of the sparsity measure."""
    _gpu()
    from engine_util import model_for, run_engine
    from golden_util import oracle_for
    from oracle.informer_np import AttnTrace

    case = load_case(name)
    m = model_for(case)
    out, dbg, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=True)
    orc = oracle_for(case)
    trace = AttnTrace()
    orc.forward(case.z["x_enc"], case.z["x_dec"], case.idx, trace=trace)
    sels = engine_selections(dbg, trace)
    trace2 = AttnTrace()
    ref, _ = orc.forward(case.z["x_enc"], case.z["x_dec"], case.idx, trace=trace2, selections=sels)
    assert rel_nmse(out, ref) < TOL
    for k, (mine, theirs) in enumerate(zip(sels, trace2.m_top)):
        M = trace2.m_val[k]                       # oracle M on the conditional trajectory
        u = mine.shape[-1]
        for b, h in zip(*np.nonzero((mine != theirs).any(-1))):
            srt = np.sort(M[b, h])[::-1]
            boundary = 0.5 * (srt[u - 1] + srt[u])
            spread = srt[0] - srt[-1]
            gap = np.abs(M[b, h][np.setxor1d(mine[b, h], theirs[b, h])] - boundary).max()
            assert gap < 0.02 * spread, (k, b, h, gap, spread)


def test_torch_global_rng_protocol():
    """torch.manual_seed(s) right before model(...) gives the reference's draws."""
    _gpu()
    from engine_util import model_for

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    torch.manual_seed(case.meta["rng_seed"])
    with torch.no_grad():
        out, attns = m(xe, range(90), xd, range(15))
    assert rel_nmse(out.cpu().numpy(), case.z["out"]) < TOL
    # a second forward continues the global stream: different draws, different output
    out2, _ = m(xe, range(90), xd, range(15))
    assert not torch.equal(out, out2)


def test_native_sampler_matches_explicit_indices():
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    ref, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    eng.seed(case.meta["rng_seed"])
    dev = torch.device("cuda:0")
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    out = torch.empty(4, 5, 16, device=dev)
    eng.forward(xe, xd, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_resident_sampler_continues_the_stream():
    """The v2 kernel replays the mt19937 stream on the device (cet_mt.hpp); forwards, host draws
    and forwards interleaved must consume exactly the draws torch.randint would, in order."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    seed = 4242
    # host mirror: the draws of forwards #1..#5 in stream order
    shapes = eng.prob_calls()
    torch.manual_seed(seed)
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in range(5)]
    eng.seed(seed)
    outs = []
    for i in range(3):                      # #1, #2, #3 on the device stream (twists cross forwards)
        o = torch.empty(4, 5, 16, device=dev)
        eng.forward(xe, xd, o)
        outs.append(o)
    got = eng.native_draw()                 # #4 drawn by the host (catches up, invalidates the device copy)
    for g, r in zip(got, draws[3]):
        np.testing.assert_array_equal(g, r)
    o5 = torch.empty(4, 5, 16, device=dev)
    eng.forward(xe, xd, o5)                 # #5: state re-uploaded from the host mirror
    torch.cuda.synchronize()
    for i, o in enumerate(outs + [o5]):
        j = i if i < 3 else 4
        ref, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], draws[j])
        np.testing.assert_array_equal(o.cpu().numpy(), ref, err_msg=f"forward #{j + 1}")


def test_prepared_tables_continue_the_stream():
    """v3 at B >= 64 stages tables prepared ahead (by the previous forward's first workgroup to
    finish, or a prep launch after a reseed).  Interleaved with small forwards (in-kernel replay,
    or the pending prepared tables) and a host draw, every forward must consume exactly the draws
    torch.randint would, in order (bitwise against explicit-index runs)."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe_np = np.ascontiguousarray(np.tile(case.z["x_enc"], (32, 1, 1)))
    xd_np = np.ascontiguousarray(np.tile(case.z["x_dec"], (32, 1, 1)))
    xe, xd = torch.from_numpy(xe_np).to(dev), torch.from_numpy(xd_np).to(dev)
    seed = 777
    shapes = eng.prob_calls()
    torch.manual_seed(seed)
    plan = [128, 128, 4, 4, 128, 0, 128, 128]   # forward batch sizes in order; 0 = a host draw
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in plan]
    eng.seed(seed)
    outs = []
    for i, B in enumerate(plan):
        if B == 0:
            for g, r in zip(eng.native_draw(), draws[i]):
                np.testing.assert_array_equal(g, r)
            outs.append(None)
            continue
        o = torch.empty(B, 5, 16, device=dev)
        eng.forward(xe[:B].contiguous(), xd[:B].contiguous(), o)
        outs.append(o)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        if o is None:
            continue
        B = o.shape[0]
        ref, _, _ = run_engine(m, xe_np[:B], xd_np[:B], draws[i])
        np.testing.assert_array_equal(o.cpu().numpy(), ref, err_msg=f"forward #{i + 1} (B={B})")


def test_device_sampler_prepared_tables_with_batches_past_one_wave():
    """Batches larger than the 512 workgroup slots (a second wave of workgroups starts while the first is still
    running) on the device-resident sampler with prepared tables: the first workgroup to finish prepares the next
    forward's tables while later workgroups of the current forward still read this one's.  Every forward must
    consume exactly torch.randint's draws — bitwise against explicit-index runs of the same batches."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe_np = np.ascontiguousarray(np.tile(case.z["x_enc"], (258, 1, 1)))   # 1,032 sequences
    xd_np = np.ascontiguousarray(np.tile(case.z["x_dec"], (258, 1, 1)))
    xe, xd = torch.from_numpy(xe_np).to(dev), torch.from_numpy(xd_np).to(dev)
    seed = 4099
    shapes = eng.prob_calls()
    torch.manual_seed(seed)
    plan = [1031, 1031, 600, 513, 1031]
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in plan]
    eng.seed(seed)
    outs = []
    for B in plan:
        o = torch.empty(B, 5, 16, device=dev)
        eng.forward(xe[:B].contiguous(), xd[:B].contiguous(), o)
        outs.append(o)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        B = o.shape[0]
        ref, _, _ = run_engine(m, xe_np[:B], xd_np[:B], draws[i])
        np.testing.assert_array_equal(o.cpu().numpy(), ref, err_msg=f"forward #{i + 1} (B={B})")


def test_host_and_device_samplers_share_the_stream():
    """cet_set_sampler switches the native draws between the device-resident mt19937 and the host
    mirror mid-stream (with prepared tables pending); every forward still consumes exactly the
    draws torch.randint would (bitwise against explicit-index runs)."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe_np = np.ascontiguousarray(np.tile(case.z["x_enc"], (32, 1, 1)))
    xd_np = np.ascontiguousarray(np.tile(case.z["x_dec"], (32, 1, 1)))
    xe, xd = torch.from_numpy(xe_np).to(dev), torch.from_numpy(xd_np).to(dev)
    seed = 31337
    shapes = eng.prob_calls()
    torch.manual_seed(seed)
    plan = [("dev", 128), ("dev", 128), ("host", 128), ("host", 4), ("dev", 128), ("host", 128), ("dev", 4)]
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in plan]
    eng.seed(seed)
    outs = []
    for where, B in plan:
        eng.set_sampler(where == "host")
        o = torch.empty(B, 5, 16, device=dev)
        eng.forward(xe[:B].contiguous(), xd[:B].contiguous(), o)
        outs.append(o)
    eng.set_sampler(False)
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        B = o.shape[0]
        ref, _, _ = run_engine(m, xe_np[:B], xd_np[:B], draws[i])
        np.testing.assert_array_equal(o.cpu().numpy(), ref, err_msg=f"forward #{i + 1} ({plan[i]})")


def test_batch_sharding_is_bitwise_per_sequence():
    """Every sequence is independent: a batch split in shards gives bitwise-identical rows."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    xe, xd, _ = make_batch(48, seed=7)
    full, _, _ = run_engine(m, xe, xd, case.idx)
    parts = [run_engine(m, xe[i:i + 16], xd[i:i + 16], case.idx)[0] for i in (0, 16, 32)]
    np.testing.assert_array_equal(np.concatenate(parts), full)


@pytest.mark.parametrize("B", [1, 37, 256, 512])
def test_random_batches_vs_oracle(B):
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from engine_util import model_for, run_engine
    from golden_util import oracle_for

    case = load_case("informer_prob_b4")
    m = model_for(case)
    xe, xd, _ = make_batch(B, seed=100 + B)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    sl = slice(max(0, B - 64), B)        # the oracle checks the last (up to) 64 rows of the launch
    ref, _ = oracle_for(case).forward(xe[sl], xd[sl], case.idx)
    assert rel_nmse(out[sl], ref) < TOL


@pytest.mark.parametrize("name,B", [("informer_lsq8", 1024), ("informer_full_e43", 512),
                                    ("informer_prob_seq48", 512), ("informer_prob_e43", 512)])
def test_full_size_production_launch_vs_oracle(name, B):
    """The production instance at full batch (C5 LSQ: B=1024; TimingAnalysis attn=full e=[4,3]: 512)
    on seeded channels; the oracle checks a 64-row slice of the launch (first and last 32 rows)."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from engine_util import model_for, run_engine
    from golden_util import oracle_for

    case = load_case(name)
    m = model_for(case)
    cfg = case.cfg
    xe, xd, _ = make_batch(B, cfg["seq_len"], cfg["label_len"], cfg["pred_len"], seed=500 + B)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    if name.endswith("_e43"):   # the e_layers [4, 3] stack takes its compile-time instance (plan_shape)
        assert m.engine(torch.device("cuda:0")).last_kernel() == E43_KERNEL
    rows = np.r_[0:32, B - 32:B]
    ref, _ = oracle_for(case).forward(xe[rows], xd[rows], case.idx)
    assert np.isfinite(out).all()
    assert rel_nmse(out[rows], ref) < TOL


@pytest.mark.parametrize("B", [1, 3, 64, 256])
def test_encoder_split_small_batches_vs_oracle(B):
    """attn="full" stacks at B·n_enc <= 512 run each encoder on its own workgroup; the last of a
    sequence's workgroups fetches the other encoders' rows of the stack output and runs the decoder
    (cet_informer4.hpp SPLIT).  Every row is checked against the oracle, and repeated launches (the
    arrival counters re-arm themselves) give identical outputs."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from engine_util import model_for, run_engine
    from golden_util import oracle_for

    case = load_case("informer_full_e43")
    m = model_for(case)
    cfg = case.cfg
    xe, xd, _ = make_batch(B, cfg["seq_len"], cfg["label_len"], cfg["pred_len"], seed=900 + B)
    out, _, _ = run_engine(m, xe, xd, case.idx)
    assert m.engine(torch.device("cuda:0")).last_kernel() == E43_SPLIT_KERNEL
    again, _, _ = run_engine(m, xe, xd, case.idx)
    np.testing.assert_array_equal(out, again)
    rows = np.arange(B) if B <= 64 else np.r_[0:32, B - 32:B]
    ref, _ = oracle_for(case).forward(xe[rows], xd[rows], case.idx)
    assert np.isfinite(out).all()
    assert rel_nmse(out[rows], ref) < TOL


@pytest.mark.parametrize("e_layers,B", [([3, 2, 1], 5), ([2, 2, 1, 1], 3), ([3, 2, 1], 170)])
def test_encoder_split_deeper_stacks_vs_oracle(e_layers, B):
    """The encoder split with three and four encoders per stack (seeded synthetic weights, attn="full")
    against the float64 oracle; at B=170 the grid is 510 workgroups."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, e_layers, 3, 64, 0.05, "full", "fixed", "gelu", False,
                      True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 3).items()})
    m.eval()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    orc = InformerOracle(InformerConfig(e_layers=tuple(e_layers), attn="full"), state)
    xe, xd, _ = make_batch(B, seed=77 + B)
    with torch.no_grad():
        # the callers' 19-positional-argument call leaves output_attention on: (out, lazy attns)
        res = m(torch.from_numpy(xe).to(dev), range(90), torch.from_numpy(xd).to(dev), range(15))
    out = (res[0] if isinstance(res, tuple) else res).cpu().numpy()
    rows = np.arange(B) if B <= 16 else np.r_[0:8, B - 8:B]
    ref, _ = orc.forward(xe[rows], xd[rows], ())
    assert np.isfinite(out).all()
    assert rel_nmse(out[rows], ref) < TOL


def test_encoder_split_e43_rows_with_dff128_vs_oracle():
    """The TimingAnalysis stack's rows (e_layers [4, 3], seq_len 90, attn "full") with d_ff 128: the
    compile-time E43 instance exists for d_ff 64 only, so this plan must take the generic encoder-split
    instance (it once got no instance at all and the forward failed).  B = 64 (split) and
    B = 300 (B·n_enc > 512: the whole-sequence generic instance), against the float64 oracle."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, [4, 3], 3, 128, 0.05, "full", "fixed", "gelu", False,
                      True, dev)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 8).items()})
    m.eval()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    orc = InformerOracle(InformerConfig(e_layers=(4, 3), d_ff=128, attn="full"), state)
    for B, kernel in ((64, "cet::v4::informer_forward_v4<128, false, 0, true, 0, false, false, 0>"),
                      (300, "cet::v4::informer_forward_v4<128, false, 0, false, 0, false, false, 0>")):
        xe, xd, _ = make_batch(B, seed=500 + B)
        with torch.no_grad():
            res = m(torch.from_numpy(xe).to(dev), range(90), torch.from_numpy(xd).to(dev), range(15))
        out = (res[0] if isinstance(res, tuple) else res).cpu().numpy()
        assert m.engine(dev).last_kernel() == kernel
        rows = np.r_[0:8, B - 8:B]
        ref, _ = orc.forward(xe[rows], xd[rows], ())
        assert np.isfinite(out).all()
        assert rel_nmse(out[rows], ref) < TOL


def test_attention_maps_materialised():
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b1")
    m = model_for(case)
    out, _, (buf, layout, per) = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, attns=True)
    for l, (off, L) in enumerate(layout):
        a = buf[off:off + 8 * L * L].reshape(8, L, L)
        ref = case.z[f"attn_e0_l{l}"]
        # rows of 1/L for unselected queries, softmax rows for the selected ones
        np.testing.assert_allclose(a.sum(-1), 1.0, atol=1e-4)
        assert rel_nmse(a, ref) < TOL, l


def test_lazy_attns_return_value():
    _gpu()
    from engine_util import model_for

    case = load_case("informer_prob_b1")
    m = model_for(case)
    dev = torch.device("cuda:0")
    torch.manual_seed(1)
    out, attns = m(torch.from_numpy(case.z["x_enc"]).to(dev), None, torch.from_numpy(case.z["x_dec"]).to(dev), None)
    assert len(attns) == 1 and len(attns[0]) == 4
    a0 = attns[0][0]
    assert tuple(a0.shape) == (1, 8, 90, 90)
    assert rel_nmse(a0.cpu().numpy()[0], case.z["attn_e0_l0"]) < TOL


@pytest.mark.parametrize("name", ["informer_prob_b1", "informer_full_e43", "informer_single_e3"])
def test_attention_maps_split_bf16(name):
    """The attns maps in split bf16 against every map the reference fixtures hold (fp32 level)."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case(name)
    m = model_for(case)
    m.engine(torch.device("cuda:0")).set_precision("split-bf16")
    _, _, (buf, layout, per) = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, attns=True)
    n = 0
    for l, (off, L) in enumerate(layout):
        key = f"attn_e0_l{l}"
        if key in case.z:
            a = buf[off:off + 8 * L * L].reshape(8, L, L)
            assert rel_nmse(a, case.z[key]) < SPLIT_TOL, (l, rel_nmse(a, case.z[key]))
            n += 1
    assert n > 0


@pytest.mark.parametrize("shape", [(300, 5, 16), (512, 5, 16), (1, 5, 16), (37, 20, 16), (64, 7, 3)])
def test_nmse_split_kernel(shape):
    """Row-owner fast path (F % 4 == 0) and the per-step fallback (F = 3), plus the running sum."""
    _gpu()
    from channelestimationtransformer_amd.engine import nmse_split
    from oracle.metrics_np import nmse_split as ref_split

    rng = np.random.default_rng(sum(shape))
    p = rng.standard_normal(shape).astype(np.float32)
    y = rng.standard_normal(shape).astype(np.float32)
    dev = torch.device("cuda:0")
    pd, yd = torch.from_numpy(p).to(dev), torch.from_numpy(y).to(dev)
    got = nmse_split(pd, yd).cpu().numpy()
    np.testing.assert_allclose(got, ref_split(p, y), rtol=1e-6)
    acc = torch.zeros(shape[1], device=dev)
    for _ in range(3):
        nmse_split(pd, yd, acc, accumulate=True)
    np.testing.assert_allclose(acc.cpu().numpy(), 3 * ref_split(p, y), rtol=1e-5)


def test_weight_reload_keeps_the_stream():
    """A weight reload while prepared tables are pending (B >= 64 after a seed) must not skip a
    forward's draws: seed, forward, reload, forward — bitwise equal to explicit-index runs."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe_np = np.ascontiguousarray(np.tile(case.z["x_enc"], (32, 1, 1)))
    xd_np = np.ascontiguousarray(np.tile(case.z["x_dec"], (32, 1, 1)))
    xe, xd = torch.from_numpy(xe_np).to(dev), torch.from_numpy(xd_np).to(dev)
    seed = 2024
    shapes = eng.prob_calls()
    torch.manual_seed(seed)
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in range(3)]
    eng.seed(seed)
    outs = []
    for i in range(3):
        o = torch.empty(128, 5, 16, device=dev)
        eng.forward(xe, xd, o)
        outs.append(o)
        if i == 0:
            # repack + re-upload the same weights with the next forward's tables pending
            eng.load_state_dict({k: np.asarray(v) for k, v in case.state.items()})
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        ref, _, _ = run_engine(m, xe_np, xd_np, draws[i])
        np.testing.assert_array_equal(o.cpu().numpy(), ref, err_msg=f"forward #{i + 1}")


def test_model_native_rng_seed_matches_torch_randint():
    """model.native_rng_seed = s: the engine's resident sampler, seeded once, consumes exactly the
    draws torch.manual_seed(s) + torch.randint would, forward after forward."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    shapes = eng.prob_calls()
    torch.manual_seed(99)
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in range(2)]
    m.native_rng_seed = 99
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    got = [m(xe, None, xd, None)[0].cpu().numpy() for _ in range(2)]
    for i in range(2):
        ref, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], draws[i])
        np.testing.assert_array_equal(got[i], ref, err_msg=f"forward #{i + 1}")


def test_lazy_attns_in_native_mode_replay_the_same_draws():
    """In native-sampler mode the lazy attns replay uses the forward's own draws (recorded before
    it) and does not move the stream: the next forward still gets draw #2."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_b1")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    shapes = eng.prob_calls()
    torch.manual_seed(7)
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in range(2)]
    m.native_rng_seed = 7
    xe = torch.from_numpy(case.z["x_enc"]).to(dev)
    xd = torch.from_numpy(case.z["x_dec"]).to(dev)
    out1, attns = m(xe, None, xd, None)
    maps = [a.cpu().numpy() for a in attns[0]]       # replay happens here
    out2, _ = m(xe, None, xd, None)
    ref1, _, (buf, layout, _) = run_engine(m, case.z["x_enc"], case.z["x_dec"], draws[0], attns=True)
    ref2, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], draws[1])
    np.testing.assert_array_equal(out1.cpu().numpy(), ref1)
    np.testing.assert_array_equal(out2.cpu().numpy(), ref2)
    for l, (off, L) in enumerate(layout):
        np.testing.assert_array_equal(maps[l][0], buf[off:off + 8 * L * L].reshape(8, L, L))


@pytest.mark.parametrize("fmt", ["pt", "json"])
def test_checkpoint_roundtrip_through_the_engine(tmp_path, fmt):
    """Weights written in the reference's formats (the .pt dict of QuantizationAwareTraining.py:305-313,
    the per-key JSON of exportWeights.py:55-70), read back, loaded with strict=False and run through the
    production kernel: the output matches the reference fixture."""
    _gpu()
    from channelestimationtransformer_amd.checkpoint import export_json, import_json, load_checkpoint, save_checkpoint
    from channelestimationtransformer_amd.informer import InformerStack
    from engine_util import run_engine

    case = load_case("informer_prob_b4")
    if fmt == "pt":
        p = str(tmp_path / "tmodel_49.pt")
        save_checkpoint(p, case.state, epoch=49, global_step=7)
        state = load_checkpoint(p)
    else:
        d = str(tmp_path / "weight_export")
        export_json(case.state, d)
        state = import_json(d)
    m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, [4], 3, 64, 0.05, "prob", "fixed", "gelu", False, True,
                      torch.device("cuda:0"))
    res = m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()}, strict=False)
    assert not res.missing_keys
    m.eval()
    out, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert rel_nmse(out, case.z["out"]) < TOL


@pytest.mark.parametrize("B,native", [(512, True), (37, False), (1, False)])
def test_fused_nmse_matches_standalone(B, native):
    """cet_forward_nmse: the forward's output is bitwise the plain forward's, and the fused NMSE_Split
    sums (last-workgroup fixed-order reduction) equal the standalone kernel's and the oracle's;
    accumulate mode adds the ratio; repeated launches give bitwise-identical sums."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.engine import nmse_split_sums
    from engine_util import model_for
    from oracle.metrics_np import nmse_split as ref_split

    case = load_case("informer_prob_b4")
    m = model_for(case)
    dev = torch.device("cuda:0")
    eng = m.engine(dev)
    xe_np, xd_np, lab_np = make_batch(B, seed=900 + B)
    xe, xd, lab = (torch.from_numpy(a).to(dev) for a in (xe_np, xd_np, lab_np))
    outs, sums = [], []
    acc = torch.zeros(5, device=dev)
    for i in range(3):
        if native:
            eng.seed(5)
        else:
            eng.set_indices(case.idx)
        o = torch.empty(B, 5, 16, device=dev)
        s = torch.zeros(2, 5, dtype=torch.float64, device=dev)
        eng.forward_nmse(xe, xd, o, lab, acc, s)
        outs.append(o)
        sums.append(s)
    if native:
        eng.seed(5)
    else:
        eng.set_indices(case.idx)
    plain = torch.empty(B, 5, 16, device=dev)
    eng.forward(xe, xd, plain)
    ref_s = torch.zeros(2, 5, dtype=torch.float64, device=dev)
    nmse_split_sums(plain, lab, ref_s)
    torch.cuda.synchronize()
    for o, s in zip(outs, sums):
        np.testing.assert_array_equal(o.cpu().numpy(), plain.cpu().numpy())
        np.testing.assert_array_equal(s.cpu().numpy(), sums[0].cpu().numpy())
    np.testing.assert_allclose(sums[0].cpu().numpy(), ref_s.cpu().numpy(), rtol=1e-6)
    r = (sums[0][0] / sums[0][1]).cpu().numpy()
    np.testing.assert_allclose(r, ref_split(plain.cpu().numpy(), lab_np), rtol=1e-5)
    np.testing.assert_allclose(acc.cpu().numpy(), 3 * r, rtol=1e-5)


@pytest.mark.parametrize("c_out", [16, 3])
def test_fused_nmse_odd_batch_and_label_width(c_out):
    """The fused NMSE_Split epilogue and its last-workgroup reduction at an odd batch, and with a label row
    (pred_len × c_out = 15 floats) that is not a whole number of 16-byte vectors: the labels are staged
    with element loads, never past the batch's last row."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.metrics_np import nmse_split as ref_split

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, c_out, 90, 10, 5, 5, 128, 8, [4], 3, 64, 0.05, "prob", "fixed", "gelu", False, True,
                      dev)
    state = synthetic_state_dict(informer_stack_spec(16, 16, c_out, 128, 8, [4], 3, 64, freq="gelu"), 3)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    eng = m.eval().engine(dev)
    eng.seed(2)
    B = 65
    xe_np, xd_np, lab_np = make_batch(B, seed=3)
    lab_np = np.ascontiguousarray(lab_np[..., :c_out])
    xe, xd, lab = (torch.from_numpy(a).to(dev) for a in (xe_np, xd_np, lab_np))
    o = torch.empty(B, 5, c_out, device=dev)
    s = torch.zeros(2, 5, dtype=torch.float64, device=dev)
    eng.forward_nmse(xe, xd, o, lab, None, s)
    torch.cuda.synchronize()
    assert eng.last_path() == "v4"
    np.testing.assert_allclose((s[0] / s[1]).cpu().numpy(), ref_split(o.cpu().numpy(), lab_np), rtol=1e-5)


# the shape instances (the last template argument: the decoder on the LDS-DMA weight feed, opt-in CET_FEED=1)
C2_KERNEL = "cet::v4::informer_forward_v4<64, false, 0, false, 1, false, false, 0>"     # plan_shape V4S_C2
E43_KERNEL = "cet::v4::informer_forward_v4<64, false, 0, false, 2, false, false, 0>"    # V4S_E43 (TimingAnalysis)
E43_SPLIT_KERNEL = "cet::v4::informer_forward_v4<64, false, 0, true, 2, false, false, 0>"


def _c2_model(attn, seed, bias_offset=0.0):
    """The C2 architecture (e_layers [4], distil, seq_len 90) with seeded synthetic weights; bias_offset is
    added to every attention out-projection bias, so every LN1 input row carries that mean offset."""
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, [4], 3, 64, 0.05, attn, "fixed", "gelu", False, True, dev)
    sd = synthetic_state_dict(m._schema(), seed)
    if bias_offset:
        sd = {k: (np.asarray(v) + np.float32(bias_offset) if k.endswith("out_projection.bias") else v)
              for k, v in sd.items()}
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.eval()


@pytest.mark.parametrize("attn", ["full", "prob"])
def test_c2_instance_on_every_plan_it_accepts(attn):
    """plan_is_c2 (cet_api.cpp) routes every plan with C2's encoder rows (one encoder, 90 → 45 → 23 → 12, the
    first three layers distilling) to the compile-time C2 instance, whatever the attention: attn="full"
    (FullAttention in every layer, attn.py:37-70; PL.prob is a runtime flag inside the instance) as well as
    "prob".  B = 512 against the float64 oracle on a row slice, and the instance asserted by name."""
    _gpu()
    from engine_util import run_engine

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.rng import draw_indices
    from oracle.informer_np import InformerConfig, InformerOracle, sample_shapes

    m = _c2_model(attn, 6)
    cfg = InformerConfig(attn=attn)
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    idx = draw_indices(sample_shapes(cfg), seed=21) if attn == "prob" else None
    xe, xd, _ = make_batch(512, seed=88)
    out, _, _ = run_engine(m, xe, xd, idx)
    eng = m.engine(torch.device("cuda:0"))
    assert eng.last_path() == "v4"
    assert eng.last_kernel() == C2_KERNEL
    rows = np.r_[0:16, 496:512]
    ref, _ = InformerOracle(cfg, state).forward(xe[rows], xd[rows], idx if idx is not None else ())
    assert rel_nmse(out[rows], ref) < TOL, rel_nmse(out[rows], ref)


@pytest.mark.parametrize("offset", [1e2, 3e2])
def test_layernorm_rows_with_a_large_mean_offset(offset):
    """LayerNorm rows whose mean is far above their spread (every attention out-projection bias shifted by
    `offset`, so each LN1 input row has mean ≈ offset and std ≈ 1): the one-pass (Σx, Σx²) statistics of
    ln_res must still meet the north star's 1e-4 against the float64 oracle (encoder.py:49-50, decoder.py:
    31-33; torch.nn.LayerNorm's biased variance).  C2 architecture, attn="full", B = 64."""
    _gpu()
    from engine_util import run_engine

    from channelestimationtransformer_amd.dataset import make_batch
    from oracle.informer_np import InformerConfig, InformerOracle

    m = _c2_model("full", 7, bias_offset=offset)
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    xe, xd, _ = make_batch(64, seed=90)
    out, _, _ = run_engine(m, xe, xd)
    assert m.engine(torch.device("cuda:0")).last_kernel() == C2_KERNEL
    ref, _ = InformerOracle(InformerConfig(attn="full"), state).forward(xe, xd, ())
    assert rel_nmse(out, ref) < TOL, rel_nmse(out, ref)


@pytest.mark.parametrize("which,B", [("c2-prob", 512), ("c2-full", 512), ("e43", 512), ("e43", 40)])
def test_decoder_feed_bitwise_equals_register_path(which, B):
    """The decoder on the LDS-DMA weight feed (opt-in CET_FEED=1, measured slower: DESIGN §3.0f; weight tiles six
    ahead in per-wave LDS slots, bias / LayerNorm vectors from a per-(layer, wave) parameter tile) computes
    exactly what the register path computes: the same bytes in the same MFMAs and epilogues.  Each plan runs on
    the register path (default) and with CET_FEED=1 (a separately built engine) on the same inputs and draws:
    outputs bitwise equal, the instances asserted by name.  C2 under both attention modes at B = 512, the TimingAnalysis stack at B = 512 and in its
    encoder-split form (B = 40)."""
    _gpu()
    import os

    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.informer import InformerStack
    from channelestimationtransformer_amd.rng import draw_indices
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from engine_util import run_engine
    from oracle.informer_np import InformerConfig, sample_shapes

    dev = torch.device("cuda:0")
    attn = "prob" if which == "c2-prob" else "full"
    e_layers = [4, 3] if which == "e43" else [4]

    def build():
        m = InformerStack(16, 16, 16, 90, 10, 5, 5, 128, 8, e_layers, 3, 64, 0.05, attn, "fixed", "gelu", False,
                          True, dev)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(m._schema(), 12).items()})
        return m.eval()

    idx = draw_indices(sample_shapes(InformerConfig(attn=attn, e_layers=tuple(e_layers))), seed=5) \
        if attn == "prob" else None
    xe, xd, _ = make_batch(B, seed=610 + B)
    m = build()
    ref, _, _ = run_engine(m, xe, xd, idx)
    name = m.engine(dev).last_kernel()
    assert name.endswith(", false, 0>"), name
    os.environ["CET_FEED"] = "1"
    try:
        m2 = build()
        out, _, _ = run_engine(m2, xe, xd, idx)
        name2 = m2.engine(dev).last_kernel()
    finally:
        del os.environ["CET_FEED"]
    assert name2 == name[:-len(", false, 0>")] + ", true, 0>", (name, name2)
    assert np.isfinite(out).all()
    np.testing.assert_array_equal(out, ref)


def test_lab20_mixed_precision_vs_reference_fixture():
    """The mixed policy (cet_set_precision 4: the encoder in bf16 at two workgroups per CU, the decoder in split
    bf16) on the genuinely sparse masked decoder (label_len 20: L_dec 25, u 20; unselected rows take cumsum(V),
    attn.py:120-125): the decoder's ProbSparse selections equal the reference's M_top in every decoder call
    (the DIAG instance's M dumps), the output is within 1e-4 of the reference's own, and the production (C2
    shape) instance agrees with the diagnostic one.  The encoder's calls run in bf16 and may swap near-tie
    queries (< 1e-5 there); they are not asserted."""
    _gpu()
    from engine_util import model_for, run_engine

    case = load_case("informer_prob_lab20")
    m = model_for(case)
    eng = m.engine(torch.device("cuda:0"))
    eng.set_precision("mixed")
    assert eng.precision() == "mixed"
    out, dbg, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx, debug=True)
    prod, _, _ = run_engine(m, case.z["x_enc"], case.z["x_dec"], case.idx)
    assert eng.last_kernel() == "cet::v4::informer_forward_v4<64, false, 0, false, 1, false, false, 1>"
    el = case.cfg["e_layers"]
    n_enc_calls = sum(el) if isinstance(el, (list, tuple)) else int(el)
    bad = 0
    for k in range(n_enc_calls, case.meta["n_mtop"]):   # the decoder's calls
        Mk = dbg[f"M{k}"]
        mt = case.z[f"mtop{k}"]
        sel = np.sort(np.argsort(-Mk, axis=-1, kind="stable")[..., :mt.shape[-1]], axis=-1)
        bad += int((sel != mt).any(-1).sum())
    assert bad == 0, bad
    assert np.isfinite(prod).all()
    assert rel_nmse(prod, case.z["out"]) < TOL, rel_nmse(prod, case.z["out"])
    assert rel_nmse(prod, out) < 1e-10, rel_nmse(prod, out)
