"""Generate tests/golden/data_seqdata.npz by running the REFERENCE's own data path.

Development container only (reads the read-only reference tree at /root/reference, absent on
the GPU box).  A SeqData instance is built around an in-memory complex64 dataset (the
reference's CDL pickles are absent); for each batch element the global RNGs are seeded, the
reference's ``SeqData.__getitem__`` (FullPrecision/dataset.py:133-152) produces
``(H, H_noise, H_seq, H_pred)`` and ``LoadBatch`` (:20-44) the model arrays; the same seeds are
then replayed to record the draws it consumed: the window start (``np.random.randint``) and the
two ``torch.randn`` arrays of ``noise`` (:54-74).  The decoder input follows the callers'
``run_validation`` (QuantizationAwareTraining.py:101-114), which cannot be imported.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_data_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/FullPrecision")

import dataset as ref  # noqa: E402  (the reference module)

SEQ, LAB, PRED, SNR = 90, 10, 5, 14.0
N_SAMPLES, SLOTS, NR, NT = 6, 100, 2, 4
IDX = [3, 0, 5, 3]


def main():
    rng = np.random.default_rng(77)
    # non-unit-power samples so channelnorm matters
    scale = rng.uniform(0.2, 3.0, size=(N_SAMPLES, 1, 1, 1))
    H = (rng.standard_normal((N_SAMPLES, SLOTS, NR, NT)) + 1j * rng.standard_normal((N_SAMPLES, SLOTS, NR, NT)))
    data = torch.from_numpy((H * scale).astype(np.complex64))

    sd = ref.SeqData.__new__(ref.SeqData)
    sd.seq_len, sd.pred_len, sd.length, sd.SNR, sd.dataset = SEQ, PRED, SEQ + PRED, SNR, data

    starts, res, ims, h_seq, h_pred = [], [], [], [], []
    for b, s in enumerate(IDX):
        np.random.seed(1000 + b)
        torch.manual_seed(2000 + b)
        _, _, hs, hp = sd[s]
        h_seq.append(np.asarray(hs))
        h_pred.append(np.asarray(hp))
        np.random.seed(1000 + b)
        starts.append(np.random.randint(0, SLOTS - (SEQ + PRED) + 1))
        torch.manual_seed(2000 + b)
        res.append(torch.randn(SLOTS, NR, NT).numpy())
        ims.append(torch.randn(SLOTS, NR, NT).numpy())
    x_enc = ref.LoadBatch(np.stack(h_seq))
    label = ref.LoadBatch(np.stack(h_pred))
    # run_validation's decoder input (QuantizationAwareTraining.py:101-114)
    x_dec = torch.cat([x_enc[:, SEQ - LAB:SEQ, :], torch.zeros_like(x_enc[:, -PRED:, :])], dim=1)
    np.savez_compressed(
        os.path.join(HERE, "data_seqdata.npz"),
        dataset=data.numpy(), idx=np.array(IDX, np.int32), starts=np.array(starts, np.int32),
        re=np.stack(res), im=np.stack(ims), snr=np.float64(SNR),
        seq_len=SEQ, label_len=LAB, pred_len=PRED,
        h_seq=np.stack(h_seq), h_pred=np.stack(h_pred),
        x_enc=x_enc.numpy(), x_dec=x_dec.numpy(), label=label.numpy())
    print("wrote data_seqdata.npz; starts", starts)


if __name__ == "__main__":
    main()
