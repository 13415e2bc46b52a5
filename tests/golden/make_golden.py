"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run only in the development container, where the read-only reference tree is at
/root/reference (it does not exist on the GPU box; nothing else in the repo reads
it).  The script imports the reference model classes, loads the seeded synthetic
state dict of ``channelestimationtransformer_amd.weights`` into them, runs the CPU
forward in eval/no_grad with ``torch.manual_seed(rng_seed)`` right before it (the
ProbSparse RNG protocol of SURVEY §8c), and records:

* inputs ``x_enc``, ``x_dec``, ``label``;
* every ``torch.randint`` result in call order (``idx0``, ``idx1``, ...);
* ``M_top`` of every ProbAttention call (sorted per (b, h): ``topk(sorted=False)``);
* per-stage activations from forward hooks (``act_*``);
* the output, the ``attns`` maps of batch element 0 (``attn_*``) and
  ``NMSELossSplit(output, label)``.

Weights are NOT stored: tests regenerate them from ``(spec, weight_seed)``.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from channelestimationtransformer_amd import spec as S  # noqa: E402
from channelestimationtransformer_amd.dataset import make_batch  # noqa: E402
from channelestimationtransformer_amd.weights import synthetic_state_dict  # noqa: E402

FP_CFG = dict(seq_len=90, label_len=10, pred_len=5, d_model=128, enc_in=16, dec_in=16, c_out=16,
              n_heads=8, e_layers=[4], d_layers=3, d_ff=64, dropout=0.05, attn="prob", embed="fixed",
              activation="gelu", output_attention=False, distil=True, factor=5)

CASES = {
    # C1: FullPrecision/config.py exactly, batch 1 (with activations + attns)
    "informer_prob_b1": dict(model="informer_stack", cfg={}, B=1, acts=True),
    "informer_prob_b4": dict(model="informer_stack", cfg={}, B=4, acts=False),
    # TimingAnalysis/config.py shapes: attn="full", e_layers=[4,3]
    "informer_full_e43": dict(model="informer_stack", cfg=dict(attn="full", e_layers=[4, 3]), B=2, acts=True),
    "informer_prob_e43": dict(model="informer_stack", cfg=dict(e_layers=[4, 3]), B=2, acts=False),
    # decoder length 25 -> u = 20 < 25: genuinely sparse decoder ProbAttention
    "informer_prob_lab20": dict(model="informer_stack", cfg=dict(label_len=20), B=2, acts=True),
    "informer_prob_seq48": dict(model="informer_stack", cfg=dict(seq_len=48), B=2, acts=False),
    # C3: build_transformer(16,16,90,5,10,128,3,8,0.05,64)
    "transformer_c3": dict(model="transformer", cfg={}, B=4, acts=True),
    # C5: LSQ 8-bit weights (models/InformerLSQ); the LSQ study sweeps 8..11 bits
    # (QuantizationStudy/LSQ/TrainInformerLSQ.py:338)
    "informer_lsq8": dict(model="informer_lsq", cfg=dict(num_bits=8), B=2, acts=False),
    "informer_lsq9": dict(model="informer_lsq", cfg=dict(num_bits=9), B=2, acts=False),
    "informer_lsq10": dict(model="informer_lsq", cfg=dict(num_bits=10), B=2, acts=False),
    "informer_lsq11": dict(model="informer_lsq", cfg=dict(num_bits=11), B=2, acts=False),
    # single-encoder Informer (FullPrecision/InformerModel/model.py:11-139), e_layers an int
    "informer_single_e3": dict(model="informer", cfg=dict(e_layers=3), B=2, acts=True),
    # shapes outside the fused kernels (the layer-wise engine): the MimoSimulation checkpoint's
    # d_model 64 with e_layers [4,3]; the TimingAnalysis sweeps' n_heads that do not divide d_model
    # (d_keys = d_model // n_heads, TrainInformer.py:236-264), d_ff and d_model beyond 128, and a
    # long, genuinely sparse decoder (label_len 25 + pred_len 9)
    "informer_d64_e43": dict(model="informer_stack", cfg=dict(d_model=64, e_layers=[4, 3]), B=2, acts=True),
    # the MimoSimulation checkpoint's own architecture (Predict.py:91-93: seq_len 25, d_model 64, e_layers
    # [4,3], attn "full"): the shape the fused layer-wise form carries
    "informer_d64_s25_full": dict(model="informer_stack", cfg=dict(d_model=64, e_layers=[4, 3], seq_len=25,
                                                                   attn="full"), B=2, acts=True),
    "informer_h5_ff256": dict(model="informer_stack", cfg=dict(n_heads=5, d_ff=256), B=2, acts=False),
    "informer_d256_h3_lab25": dict(model="informer_stack",
                                   cfg=dict(d_model=256, n_heads=3, d_ff=128, seq_len=48, label_len=25, pred_len=9),
                                   B=2, acts=False),
    "informer_full_d512_h4": dict(model="informer_stack",
                                  cfg=dict(attn="full", d_model=512, n_heads=4, d_ff=512, e_layers=[2], d_layers=1,
                                           seq_len=24, label_len=8, pred_len=3),
                                  B=2, acts=True),
}


def _informer_schema(cfg, lsq=False):
    return S.informer_stack_spec(cfg["enc_in"], cfg["dec_in"], cfg["c_out"], cfg["d_model"], cfg["n_heads"],
                                 cfg["e_layers"], cfg["d_layers"], cfg["d_ff"], embed=cfg["embed"],
                                 freq=cfg["activation"], distil=True, lsq=lsq)


def build_reference(kind, cfg):
    dev = torch.device("cpu")
    if kind == "informer_stack":
        sys.path.insert(0, os.path.join(REF, "FullPrecision"))
        from InformerModel.model import InformerStack
        # the callers' 19-positional-argument call (QuantizationAwareTraining.py:63-83)
        m = InformerStack(cfg["enc_in"], cfg["dec_in"], cfg["c_out"], cfg["seq_len"], cfg["label_len"],
                          cfg["pred_len"], cfg["factor"], cfg["d_model"], cfg["n_heads"], cfg["e_layers"],
                          cfg["d_layers"], cfg["d_ff"], cfg["dropout"], cfg["attn"], cfg["embed"],
                          cfg["activation"], cfg["output_attention"], cfg["distil"], dev)
        return m, _informer_schema(cfg)
    if kind == "informer":
        sys.path.insert(0, os.path.join(REF, "FullPrecision"))
        from InformerModel.model import Informer
        m = Informer(cfg["enc_in"], cfg["dec_in"], cfg["c_out"], cfg["seq_len"], cfg["label_len"],
                     cfg["pred_len"], cfg["factor"], cfg["d_model"], cfg["n_heads"], cfg["e_layers"],
                     cfg["d_layers"], cfg["d_ff"], cfg["dropout"], cfg["attn"], cfg["embed"],
                     cfg["activation"], cfg["output_attention"], cfg["distil"], dev)
        return m, S.informer_spec(cfg["enc_in"], cfg["dec_in"], cfg["c_out"], cfg["d_model"], cfg["n_heads"],
                                  cfg["e_layers"], cfg["d_layers"], cfg["d_ff"], embed=cfg["embed"],
                                  freq=cfg["activation"], distil=True)
    if kind == "informer_lsq":
        sys.path.insert(0, REF)
        from models.InformerLSQ.model import InformerStack
        from models.InformerLSQ.LSQ import LinearLSQ, Conv1dLSQ
        # TrainInformerLSQ.py:80-101: a 20th positional argument (num_bits) lands in `mix`
        m = InformerStack(cfg["enc_in"], cfg["dec_in"], cfg["c_out"], cfg["seq_len"], cfg["label_len"],
                          cfg["pred_len"], cfg["factor"], cfg["d_model"], cfg["n_heads"], cfg["e_layers"],
                          cfg["d_layers"], cfg["d_ff"], cfg["dropout"], cfg["attn"], cfg["embed"],
                          cfg["activation"], cfg["output_attention"], cfg["distil"], dev, cfg["num_bits"])
        return m, _informer_schema(cfg, lsq=True)
    if kind == "transformer":
        sys.path.insert(0, REF)
        from models.Transformer.model import build_transformer
        m = build_transformer(16, 16, cfg["seq_len"], cfg["pred_len"], cfg["label_len"], cfg["d_model"],
                              cfg["d_layers"], cfg["n_heads"], cfg["dropout"], cfg["d_ff"])
        return m, S.transformer_spec(16, 16, cfg["seq_len"], cfg["pred_len"], cfg["label_len"], cfg["d_model"],
                                     cfg["d_layers"], cfg["n_heads"], cfg["d_ff"])
    raise ValueError(kind)


def lsq_enable(model, nbits, state):
    """TrainInformerLSQ.py:104-116, then load the recipe weights + step sizes."""
    from models.InformerLSQ.LSQ import LinearLSQ, Conv1dLSQ
    for _, mod in model.named_modules():
        if isinstance(mod, (LinearLSQ, Conv1dLSQ)):
            mod.quantize = True
            mod.nbits = int(nbits)
            mod.reset_parameters()


def run_case(name, c):
    cfg = dict(FP_CFG)
    cfg.update(c["cfg"])
    kind = c["model"]
    model, schema = build_reference(kind, cfg)
    weight_seed = 0
    state = synthetic_state_dict(schema, seed=weight_seed, lsq_bits=cfg.get("num_bits", 8))
    if kind == "informer_lsq":
        lsq_enable(model, cfg["num_bits"], state)
    ref_keys = list(model.state_dict().keys())
    assert ref_keys == [k for k, _, _ in schema], (name, set(ref_keys) ^ {k for k, _, _ in schema})
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()}, strict=True)
    model.eval()

    B = c["B"]
    x_enc, x_dec, label = make_batch(B, cfg["seq_len"], cfg["label_len"], cfg["pred_len"], snr=20.0, seed=1234)

    acts, mtops = {}, []
    hooks = []

    def hook(tag, pick=None):
        def f(_m, _i, out):
            o = out[0] if pick == 0 else out
            acts[tag] = o.detach().numpy().astype(np.float32)
        return f

    if kind == "informer":
        mods = dict(model.named_modules())
        hooks.append(model.enc_embedding.register_forward_hook(hook("enc_emb")))
        enc = model.encoder
        for l, lay in enumerate(enc.attn_layers):
            hooks.append(lay.register_forward_hook(hook(f"enc0_layer{l}", 0)))
        if enc.conv_layers is not None:
            for l, cl in enumerate(enc.conv_layers):
                hooks.append(cl.register_forward_hook(hook(f"enc0_conv{l}")))
        hooks.append(enc.register_forward_hook(hook("enc0_out", 0)))
        hooks.append(model.dec_embedding.register_forward_hook(hook("dec_emb")))
        for l, lay in enumerate(model.decoder.layers):
            hooks.append(lay.register_forward_hook(hook(f"dec_layer{l}")))
        hooks.append(model.decoder.register_forward_hook(hook("dec_out")))
        hooks.append(model.projection.register_forward_hook(hook("proj")))
    if kind in ("informer_stack", "informer_lsq"):
        mods = dict(model.named_modules())
        hooks.append(model.enc_embedding.register_forward_hook(hook("enc_emb")))
        for i, enc in enumerate(model.encoder.encoders):
            for l, lay in enumerate(enc.attn_layers):
                hooks.append(lay.register_forward_hook(hook(f"enc{i}_layer{l}", 0)))
            if enc.conv_layers is not None:
                for l, cl in enumerate(enc.conv_layers):
                    hooks.append(cl.register_forward_hook(hook(f"enc{i}_conv{l}")))
            hooks.append(enc.register_forward_hook(hook(f"enc{i}_out", 0)))
        hooks.append(model.encoder.register_forward_hook(hook("enc_out", 0)))
        hooks.append(model.dec_embedding.register_forward_hook(hook("dec_emb")))
        for l, lay in enumerate(model.decoder.layers):
            hooks.append(lay.register_forward_hook(hook(f"dec_layer{l}")))
        hooks.append(model.decoder.register_forward_hook(hook("dec_out")))
        hooks.append(model.projection.register_forward_hook(hook("proj")))
    if kind != "transformer":
        for n, mod in mods.items():
            if type(mod).__name__ == "ProbAttention":
                orig = mod._prob_QK

                def wrapped(Q, K, sample_k, n_top, _orig=orig):
                    qk, mt = _orig(Q, K, sample_k, n_top)
                    mtops.append(np.sort(mt.numpy(), axis=-1).astype(np.int32))
                    return qk, mt
                mod._prob_QK = wrapped
    if kind == "transformer":
        hooks.append(model.src_pos.register_forward_hook(hook("enc_emb")))
        for l, lay in enumerate(model.encoder.layers):
            hooks.append(lay.register_forward_hook(hook(f"enc_layer{l}")))
        hooks.append(model.encoder.register_forward_hook(hook("enc_out")))
        hooks.append(model.tgt_pos.register_forward_hook(hook("dec_emb")))
        for l, lay in enumerate(model.decoder.layers):
            hooks.append(lay.register_forward_hook(hook(f"dec_layer{l}")))
        hooks.append(model.decoder.register_forward_hook(hook("dec_out")))
        hooks.append(model.projection_layer.register_forward_hook(hook("proj")))

    rec = []
    orig_randint = torch.randint

    def rec_randint(*a, **k):
        r = orig_randint(*a, **k)
        rec.append(r.clone())
        return r

    rng_seed = 1
    torch.randint = rec_randint
    try:
        torch.manual_seed(rng_seed)
        with torch.no_grad():
            xe, xd = torch.from_numpy(x_enc), torch.from_numpy(x_dec)
            if kind == "transformer":
                out = model(xe, xd)
                attns = None
            else:
                out, attns = model(xe, range(cfg["seq_len"]), xd, range(cfg["pred_len"] + cfg["label_len"]))
    finally:
        torch.randint = orig_randint
        for h in hooks:
            h.remove()

    sys.path.insert(0, os.path.join(REF, "FullPrecision"))
    from metrics import NMSELossSplit
    nmse = NMSELossSplit()(out, torch.from_numpy(label)).numpy()

    res = {"x_enc": x_enc, "x_dec": x_dec, "label": label, "out": out.numpy().astype(np.float32),
           "nmse_split": nmse.astype(np.float32)}
    for k, r in enumerate(rec):
        res[f"idx{k}"] = r.numpy().astype(np.int32)
    for k, m in enumerate(mtops):
        res[f"mtop{k}"] = m
    if c["acts"]:
        for k, v in acts.items():
            res[f"act_{k}"] = v
        if attns is not None:
            if kind == "informer":          # Informer returns one encoder's per-layer maps
                attns = [attns]
            for i, enc_attns in enumerate(attns):
                for l, a in enumerate(enc_attns):
                    if a is not None:
                        res[f"attn_e{i}_l{l}"] = a[0].numpy().astype(np.float32)
    meta = dict(case=name, model=kind, cfg=cfg, B=B, weight_seed=weight_seed, rng_seed=rng_seed,
                data_seed=1234, snr=20.0, n_randint=len(rec), n_mtop=len(mtops),
                keys=[[k, list(s), kd] for k, s, kd in schema])
    res["meta"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **res)
    print(f"{name}: {os.path.getsize(path) / 1024:.0f} KiB, randint calls {len(rec)}, nmse {nmse}")


if __name__ == "__main__":
    only = sys.argv[1:]
    cwd = os.getcwd()
    os.chdir("/tmp")  # the reference tree is read-only; keep any stray output out of the repo
    try:
        for n, c in CASES.items():
            if not only or n in only:
                run_case(n, c)
    finally:
        os.chdir(cwd)
