"""Device channel pipeline (cet_prepare_batch / cet_synth_channels) against the data oracle."""
import numpy as np
import pytest
import torch

from golden_util import GOLDEN

pytestmark = pytest.mark.gpu

Z = np.load(f"{GOLDEN}/data_seqdata.npz")
TOL = 2e-6   # fp32 rounding of the two power means, relative to the array's max magnitude


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _close(got, ref, tol=TOL):
    got = got.cpu().numpy() if hasattr(got, "cpu") else got
    np.testing.assert_allclose(got, ref, rtol=0, atol=tol * np.abs(ref).max())


def _data(dataset=None, **kw):
    from channelestimationtransformer_amd.pipeline import DeviceSeqData

    return DeviceSeqData(Z["dataset"] if dataset is None else dataset, int(Z["seq_len"]), int(Z["pred_len"]),
                         SNR=float(Z["snr"]), label_len=int(Z["label_len"]), device=torch.device("cuda:0"), **kw)


def test_prepare_batch_matches_reference_seqdata():
    """Parity mode: the reference's own draws → the reference's own LoadBatch outputs."""
    _gpu()
    d = _data()
    noise = np.stack([Z["re"], Z["im"]], axis=-1)
    x_enc, x_dec, label = d.batch(idx=Z["idx"], starts=Z["starts"], noise=noise)
    torch.cuda.synchronize()
    _close(x_enc, Z["x_enc"])
    _close(x_dec, Z["x_dec"])
    _close(label, Z["label"])


def test_reference_rng_protocol_end_to_end():
    """reference_batch draws from the global generators exactly as __getitem__ would."""
    _gpu()
    d = _data()
    for b, s in enumerate(Z["idx"]):
        np.random.seed(1000 + b)
        torch.manual_seed(2000 + b)
        x_enc, x_dec, label = d.reference_batch([s])
        _close(x_enc[0], Z["x_enc"][b])
        _close(label[0], Z["label"][b])


def test_device_draws_are_deterministic_in_range_and_normal():
    _gpu()
    from oracle.data_np import get_item

    rng = np.random.default_rng(3)
    n, slots = 64, 100
    data = (rng.standard_normal((n, slots, 2, 4)) + 1j * rng.standard_normal((n, slots, 2, 4))) * 1.7
    d = _data(data)
    a = d.batch(B=n, seed=11, counter=5, return_starts=True)
    b = d.batch(B=n, seed=11, counter=5, return_starts=True)
    c = d.batch(B=n, seed=11, counter=6, return_starts=True)
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    assert not torch.equal(a[0], c[0])
    st = a[3].cpu().numpy()
    L = d.length
    assert st.min() >= 0 and st.max() <= slots - L and len(np.unique(st)) > 1
    # implied noise = x_enc − clean window: zero mean, variance sigma·(mean power = 1)
    seq = d.seq_len
    clean = np.stack([get_item(data[i], int(st[i]), np.zeros((slots, 2, 4)), np.zeros((slots, 2, 4)), d.SNR, seq,
                               d.pred_len)[2] for i in range(n)])
    from oracle.data_np import load_batch

    z = a[0].cpu().numpy().astype(np.float64) - load_batch(clean)
    sigma = 10 ** (-d.SNR / 10)
    assert abs(z.mean()) < 0.01 * np.sqrt(sigma)
    assert abs(z.var() / (sigma / 2) - 1.0) < 0.03
    # labels and decoder inputs stay clean / structured
    _close(a[2], load_batch(np.stack([get_item(data[i], int(st[i]), np.zeros((slots, 2, 4)), np.zeros((slots, 2, 4)),
                                               d.SNR, seq, d.pred_len)[3] for i in range(n)])))
    np.testing.assert_array_equal(a[1][:, d.label_len:].cpu().numpy(), 0.0)
    assert torch.equal(a[1][:, :d.label_len], a[0][:, seq - d.label_len:])


def test_out_of_range_sample_gives_nan_rows_not_a_fault():
    _gpu()
    d = _data()
    x_enc, x_dec, label = d.batch(idx=[0, 99, 2], starts=[0, 0, 1000])
    torch.cuda.synchronize()
    assert torch.isfinite(x_enc[0]).all()
    assert torch.isnan(x_enc[1]).all() and torch.isnan(label[1]).all()
    assert torch.isnan(x_enc[2]).all() and torch.isnan(x_dec[2]).all()


def test_synth_channels_match_oracle():
    _gpu()
    from channelestimationtransformer_amd.pipeline import synth_channels
    from oracle.data_np import jakes

    n, slots, paths, seed, fd = 5, 100, 16, 9, 0.02
    H = synth_channels(n, slots, seed=seed, doppler=fd, paths=paths, device=torch.device("cuda:0"))
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    alpha = rng.uniform(0, 2 * np.pi, size=(n, 8, paths)).astype(np.float32)
    phi = rng.uniform(0, 2 * np.pi, size=(n, 8, paths)).astype(np.float32)
    g = ((rng.standard_normal((n, 8, paths)) + 1j * rng.standard_normal((n, 8, paths))) / np.sqrt(2)).astype(np.complex64)
    ref = jakes(alpha, phi, g, slots, fd).reshape(n, slots, 2, 4)
    got = H.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5)


def test_pipeline_feeds_the_engine():
    """Device batch → fused forward → NMSE: the same numbers as feeding the host-restated batch."""
    _gpu()
    from channelestimationtransformer_amd.engine import nmse_split
    from engine_util import model_for, run_engine
    from golden_util import load_case
    from oracle.data_np import prepare_batch

    case = load_case("informer_prob_b4")
    m = model_for(case)
    d = _data()
    noise = np.stack([Z["re"], Z["im"]], axis=-1)
    x_enc, x_dec, label = d.batch(idx=Z["idx"], starts=Z["starts"], noise=noise)
    out_dev, _, _ = run_engine(m, x_enc.cpu().numpy(), x_dec.cpu().numpy(), case.idx)
    xe, xd, lb = prepare_batch(Z["dataset"], Z["idx"], Z["starts"], Z["re"], Z["im"], float(Z["snr"]),
                               int(Z["seq_len"]), int(Z["label_len"]), int(Z["pred_len"]))
    out_host, _, _ = run_engine(m, xe.astype(np.float32), xd.astype(np.float32), case.idx)
    np.testing.assert_allclose(out_dev, out_host, rtol=0, atol=1e-3 * np.abs(out_host).max())
    r = nmse_split(torch.from_numpy(out_dev).cuda(), label).cpu().numpy()
    assert np.all(np.isfinite(r)) and r.shape == (5,)


def test_snr_sweep_driver_runs_and_is_deterministic():
    _gpu()
    from channelestimationtransformer_amd.sweep import run_sweep

    dev = torch.device("cuda:0")
    a = list(run_sweep([12, 20], batch=64, batches=2, device=dev))
    b = list(run_sweep([12, 20], batch=64, batches=2, device=dev))
    assert [r["snr"] for r in a] == [12, 20]
    for r, s in zip(a, b):
        assert r["batches"] == 2 and r["sequences"] == 128 and len(r["nmse_db"]) == 5
        assert np.all(np.isfinite(r["nmse"]))
        assert r["nmse"] == s["nmse"]


def test_latency_mode_runs_the_timing_config():
    _gpu()
    from channelestimationtransformer_amd.latency import CONFIG, measure

    r = measure(dict(CONFIG), torch.device("cuda:0"), reps=30, warmup=3)
    assert r["reps"] == 29 and 0 < r["p50_ms"] < 50


def _c2_oracle():
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from oracle.informer_np import InformerConfig, InformerOracle

    return InformerOracle(InformerConfig(), synthetic_state_dict(
        informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu"), 0))


def test_snr_sweep_c4_batches_vs_oracle():
    """Config C4's sweep at its per-rank batch (512) for SNR 12 and 20, two batches each: the reported
    NMSE per step is the mean of per-batch NMSE_Split ratios over the engine's own predictions
    (run_validation, QuantizationAwareTraining.py:122,138; metrics.py:26-30), and a 64-row slice of every
    batch's predictions matches the float64 oracle forward with that forward's own draws (the native
    stream seeded with 1 + seed, one forward's worth per batch, torch.randint order)."""
    _gpu()
    from channelestimationtransformer_amd.sweep import run_sweep
    from golden_util import rel_nmse
    from oracle.informer_np import InformerConfig, sample_shapes
    from oracle.metrics_np import nmse_split as ref_split

    dev = torch.device("cuda:0")
    seen = []

    def cap(snr, i, xe, xd, out, lb):
        seen.append((snr, i, xe.cpu().numpy(), xd.cpu().numpy(), out.cpu().numpy(), lb.cpu().numpy()))

    res = list(run_sweep([12, 20], batch=512, batches=2, seed=0, device=dev, capture=cap))
    assert [r["snr"] for r in res] == [12, 20] and all(r["batches"] == 2 and r["sequences"] == 1024 for r in res)
    assert all(r["kernel_path"] == "v4" for r in res)
    torch.manual_seed(1)
    shapes = sample_shapes(InformerConfig())
    draws = [[torch.randint(lk, shp).numpy() for lk, shp in shapes] for _ in range(len(seen))]
    orc = _c2_oracle()
    rows = np.r_[0:32, 480:512]
    for r in res:
        mine = [x for x in seen if x[0] == r["snr"]]
        ref = np.mean([ref_split(out, lb) for _, _, _, _, out, lb in mine], axis=0)
        np.testing.assert_allclose(r["nmse"], ref, rtol=1e-6)
    for j, (snr, i, xe, xd, out, _) in enumerate(seen):
        ref, _ = orc.forward(xe[rows], xd[rows], draws[j])
        assert rel_nmse(out[rows], ref) < 1e-4, (snr, i)


def test_c4_global_batch_sharded_equals_unsharded():
    """Config C4's 4096-sequence global batch on one GPU, once unsharded and once as 8 sequential shards
    of 512 (the 8 ranks' shards, same ProbSparse draws): every sequence's prediction is bitwise equal,
    and the shards' NMSE_Split sums, added as the all_reduce adds them and collated by the sweep's own
    collate_step_sums / check_gathered_nmse, give the unsharded batch's NMSE."""
    _gpu()
    from channelestimationtransformer_amd.dataset import make_batch
    from channelestimationtransformer_amd.engine import nmse_split
    from channelestimationtransformer_amd.rng import draw_indices
    from channelestimationtransformer_amd.sharding import check_gathered_nmse, collate_step_sums
    from channelestimationtransformer_amd.sweep import build_model

    dev = torch.device("cuda:0")
    eng = build_model(dev).engine(dev)
    shapes = eng.prob_calls()
    idx = draw_indices(shapes, seed=31)
    G, W, T = 4096, 8, 5
    xe_np, xd_np, lab_np = make_batch(G, snr=16, seed=4242)
    xe, xd, lab = (torch.from_numpy(a).to(dev) for a in (xe_np, xd_np, lab_np))
    full = torch.empty(G, T, 16, device=dev)
    s_full = torch.zeros(1, 2, T, dtype=torch.float64, device=dev)
    eng.set_indices(idx)
    eng.forward_nmse(xe, xd, full, lab, None, s_full[0])
    assert eng.last_path() == "v4"
    shard = torch.empty(G, T, 16, device=dev)
    s_rank = torch.zeros(W, 2, T, dtype=torch.float64, device=dev)
    n = G // W
    for r in range(W):
        sl = slice(r * n, (r + 1) * n)
        eng.set_indices(idx)
        eng.forward_nmse(xe[sl], xd[sl], shard[sl], lab[sl], None, s_rank[r])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(shard.cpu().numpy(), full.cpu().numpy())
    ratios, nmse = collate_step_sums(s_rank.sum(0, keepdim=True), 1)   # the all_reduce's sum, one step
    ratios_full, _ = collate_step_sums(s_full, 1)
    np.testing.assert_allclose(ratios.cpu().numpy(), ratios_full.cpu().numpy(), rtol=1e-12)
    assert check_gathered_nmse(nmse_split(shard, lab), ratios[-1]) < 1e-5
