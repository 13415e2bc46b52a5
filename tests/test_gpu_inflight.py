"""Parity of the benchmarked execution mode: two engine replicas with batches in flight on two streams.

bench.py's number of record runs step k on lane k mod 2, each lane an engine replica (same weights)
with its own non-default HIP stream, inputs, resident sampler chain (seeded 1 and 2) and fused-NMSE
ticket (bench.py `lanes`).  The two launches overlap on the GPU.  Each lane's per-step outputs and fp64
NMSE_Split sums must be bitwise what the same lane gives when it runs alone and serially, and a
64-sequence slice of one step per lane must match the oracle forward with that step's draws.
Reference: FullPrecision/QuantizationAwareTraining.py:115-122 (forward + NMSELossSplit per batch),
FullPrecision/metrics.py:26-30.  Tolerance: the north star's 1e-4 relative NMSE.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, T, STEPS, NL = 512, 5, 8, 2
TOL = 1e-4


def _lanes(dev, streams):
    import bench
    from channelestimationtransformer_amd.dataset import make_batch

    lanes = []
    for i in range(NL):
        m = bench.build_model(dev)
        eng = m.engine(dev)
        eng.seed(1 + i)
        xe_np, xd_np, lab_np = make_batch(B, snr=20.0, seed=1234 + 104729 * i)
        xe, xd, lab = (torch.from_numpy(a).to(dev) for a in (xe_np, xd_np, lab_np))
        outs = [torch.full((B, T, 16), float("nan"), device=dev) for _ in range(STEPS)]
        sums = torch.full((STEPS, 2, T), float("nan"), dtype=torch.float64, device=dev)
        st = streams[i]
        # one bound step per (lane, step): every step writes its own output buffer, nothing else is enqueued
        steps = [eng.bind_forward_nmse(xe, xd, outs[k], lab, sums, st.cuda_stream) for k in range(STEPS)]
        lanes.append(dict(model=m, eng=eng, xe_np=xe_np, xd_np=xd_np, lab_np=lab_np, outs=outs, sums=sums,
                          steps=steps, stream=st))
    return lanes


def test_two_lanes_in_flight_equal_serial_lanes_and_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from channelestimationtransformer_amd.spec import informer_stack_spec
    from channelestimationtransformer_amd.weights import synthetic_state_dict
    from golden_util import rel_nmse
    from oracle.informer_np import InformerConfig, InformerOracle
    from oracle.metrics_np import nmse_split as ref_split

    dev = torch.device("cuda:0")
    # ---- the benchmarked mode: interleaved steps on two non-default streams, launches overlapping
    streams = [torch.cuda.Stream(dev) for _ in range(NL)]
    conc = _lanes(dev, streams)
    torch.cuda.synchronize(dev)
    for k in range(NL * STEPS):
        ln = conc[k % NL]
        ln["steps"][k // NL](k // NL)
    torch.cuda.synchronize(dev)
    for ln in conc:
        assert ln["eng"].last_path() == "v4"

    # ---- the same lanes alone, serially, on the default stream, with the step's draws peeked for the oracle
    ser = _lanes(dev, [torch.cuda.current_stream(dev)] * NL)
    draws = {}
    for i, ln in enumerate(ser):
        for k in range(STEPS):
            if k == 3:
                draws[i] = ln["eng"].peek_draw()
            ln["steps"][k](k)
            torch.cuda.synchronize(dev)

    for i in range(NL):
        a, s = conc[i], ser[i]
        for k in range(STEPS):
            np.testing.assert_array_equal(a["outs"][k].cpu().numpy(), s["outs"][k].cpu().numpy(),
                                          err_msg=f"lane {i} step {k}: outputs differ from the serial run")
        np.testing.assert_array_equal(a["sums"].cpu().numpy(), s["sums"].cpu().numpy(),
                                      err_msg=f"lane {i}: fp64 NMSE sums differ from the serial run")
        # the fused sums are the batch's NMSE_Split of that step's own output
        o3 = a["outs"][3].cpu().numpy()
        r = (a["sums"][3, 0] / a["sums"][3, 1]).cpu().numpy()
        np.testing.assert_allclose(r, ref_split(o3, a["lab_np"]), rtol=1e-5)
        # successive steps consume fresh draws: outputs change from step to step
        assert not np.array_equal(a["outs"][2].cpu().numpy(), o3)

    # ---- a 64-sequence slice of step 3 of each lane against the oracle with that step's draws
    oracle = InformerOracle(InformerConfig(), synthetic_state_dict(
        informer_stack_spec(16, 16, 16, 128, 8, [4], 3, 64, freq="gelu"), 0))
    for i in range(NL):
        a = conc[i]
        sl = slice(64 * i, 64 * i + 64)
        ref, _ = oracle.forward(a["xe_np"][sl], a["xd_np"][sl], draws[i])
        e = rel_nmse(a["outs"][3].cpu().numpy()[sl], ref)
        assert e < TOL, (i, e)
