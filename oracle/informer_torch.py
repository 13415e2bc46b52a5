"""CPU ORACLE (test infrastructure only) — torch-op restatement of the reference's
InformerStack / Informer inference forward, op for op as the reference runs it on the CPU.

Why a second restatement: ``bench.py``'s ``cpu_baseline`` must stand for the reference's own
PyTorch CPU path (``.eval()``, ``no_grad``, the aten ops of
``FullPrecision/InformerModel/*.py`` on all physical cores).  The numpy oracle
(:mod:`oracle.informer_np`) is the float64 checker; this module uses the same aten kernels the
reference calls (``F.linear``, circular ``F.conv1d``, the ``K_sample`` gather of ``_prob_QK``,
``topk``, ``F.layer_norm``, ``F.gelu``, BatchNorm eval, ``F.elu``, ``F.max_pool1d``), so its CPU
time is the reference's CPU time.  It is pinned to the reference-generated fixtures at
rel-NMSE < 1e-10 in float64 (``tests/test_oracle_golden.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product path never does.  ProbSparse draws are inputs (``idx``, ``torch.randint`` call
order) instead of the global generator, so the oracle is deterministic.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .informer_np import InformerConfig, lsq_quantize, u_part


class TorchInformer:
    """``InformerStack`` / ``Informer`` forward (FullPrecision/InformerModel/model.py:11-139, 142-271)."""

    def __init__(self, cfg: InformerConfig, state: Dict[str, np.ndarray], dtype=torch.float32):
        self.cfg = cfg
        self.dt = dtype
        p = {}
        for k, v in state.items():
            if k.endswith("step_size") or k.endswith("num_batches_tracked"):
                continue
            p[k] = np.asarray(v, dtype=np.float32)
        if cfg.lsq_bits is not None:          # models/InformerLSQ/LSQ.py:65-74, 305-314
            for k, v in state.items():
                if k.endswith("step_size"):
                    wk = k[: -len("step_size")] + "weight"
                    p[wk] = lsq_quantize(p[wk], np.asarray(v), cfg.lsq_bits)
        self.p = {k: torch.from_numpy(v).to(dtype) for k, v in p.items()}

    # ---------------------------------------------------------------- blocks
    def _act(self, x):
        return F.relu(x) if self.cfg.activation == "relu" else F.gelu(x)      # encoder.py:41

    def embed(self, prefix, x):
        """DataEmbedding (embed.py:132-135): TokenEmbedding circular conv (:30-49) + pe[:L]."""
        p = self.p
        y = F.conv1d(F.pad(x.permute(0, 2, 1), (1, 1), mode="circular"),
                     p[f"{prefix}.value_embedding.tokenConv.weight"], p[f"{prefix}.value_embedding.tokenConv.bias"])
        return y.transpose(1, 2) + p[f"{prefix}.position_embedding.pe"][:, : x.shape[1]]

    def prob_attention(self, q, k, v, idx, mask_flag, out_attn):
        """ProbAttention.forward (attn.py:148-175) with _prob_QK (:89-114) and the context updates (:116-146)."""
        B, LQ, H, E = q.shape
        LK = k.shape[1]
        Q, K, V = q.transpose(2, 1), k.transpose(2, 1), v.transpose(2, 1)
        U = u_part(self.cfg.factor, LK)
        u = u_part(self.cfg.factor, LQ)
        index_sample = torch.as_tensor(np.asarray(idx), dtype=torch.long)          # attn.py:96-98
        K_expand = K.unsqueeze(-3).expand(B, H, LQ, LK, E)
        K_sample = K_expand[:, :, torch.arange(LQ).unsqueeze(1), index_sample, :]
        Q_K_sample = torch.matmul(Q.unsqueeze(-2), K_sample.transpose(-2, -1)).squeeze(-2)
        M = Q_K_sample.max(-1)[0] - torch.div(Q_K_sample.sum(-1), LK)
        M_top = M.topk(u, sorted=False)[1]                                          # attn.py:105-106
        Q_reduce = Q[torch.arange(B)[:, None, None], torch.arange(H)[None, :, None], M_top, :]
        scores = torch.matmul(Q_reduce, K.transpose(-2, -1)) * (1.0 / math.sqrt(E))
        if not mask_flag:                                                           # attn.py:116-125
            context = V.mean(dim=-2).unsqueeze(-2).expand(B, H, LQ, V.shape[-1]).clone()
        else:
            context = V.cumsum(dim=-2)
        if mask_flag:                                                               # ProbMask, attn.py:23-34
            _mask = torch.ones(LQ, LK, dtype=torch.bool).triu(1)
            indicator = _mask[None, None, :].expand(B, H, LQ, LK)[
                torch.arange(B)[:, None, None], torch.arange(H)[None, :, None], M_top, :]
            scores = scores.masked_fill(indicator, -np.inf)
        attn = torch.softmax(scores, dim=-1)
        bi, hi = torch.arange(B)[:, None, None], torch.arange(H)[None, :, None]
        context[bi, hi, M_top, :] = torch.matmul(attn, V).type_as(context)         # attn.py:136-138
        attns = None
        if out_attn:                                                                # attn.py:139-144
            attns = (torch.ones(B, H, LK, LK) / LK).type_as(attn)
            attns[bi, hi, M_top, :] = attn
        return context.transpose(2, 1).contiguous(), attns

    def full_attention(self, q, k, v, mask_flag):
        """FullAttention.forward (attn.py:52-70)."""
        B, L, H, E = q.shape
        scores = torch.einsum("blhe,bshe->bhls", q, k)
        if mask_flag:
            scores = scores.masked_fill(torch.ones(L, k.shape[1], dtype=torch.bool).triu(1), -np.inf)
        A = torch.softmax(scores * (1.0 / math.sqrt(E)), dim=-1)
        return torch.einsum("bhls,bshd->blhd", A, v).contiguous()

    def attention_layer(self, prefix, xq, xkv, kind, mask_flag, mix, idx_iter, out_attn):
        """AttentionLayer.forward (attn.py:195-209), mix scramble (:205-207)."""
        p, H = self.p, self.cfg.n_heads
        B, L, _ = xq.shape
        S = xkv.shape[1]
        q = F.linear(xq, p[f"{prefix}.query_projection.weight"], p[f"{prefix}.query_projection.bias"]).view(B, L, H, -1)
        k = F.linear(xkv, p[f"{prefix}.key_projection.weight"], p[f"{prefix}.key_projection.bias"]).view(B, S, H, -1)
        v = F.linear(xkv, p[f"{prefix}.value_projection.weight"], p[f"{prefix}.value_projection.bias"]).view(B, S, H, -1)
        attn = None
        if kind == "prob":
            out, attn = self.prob_attention(q, k, v, next(idx_iter), mask_flag, out_attn)
        else:
            out = self.full_attention(q, k, v, mask_flag)
        if mix:
            out = out.transpose(2, 1).contiguous()
        out = out.view(B, L, -1)
        return F.linear(out, p[f"{prefix}.out_projection.weight"], p[f"{prefix}.out_projection.bias"]), attn

    def ffn(self, prefix, x):
        """conv1/conv2 (k=1) on x.transpose(-1, 1) (encoder.py:52-54, decoder.py:37-38)."""
        p = self.p
        y = self._act(F.conv1d(x.transpose(-1, 1), p[f"{prefix}.conv1.weight"], p[f"{prefix}.conv1.bias"]))
        return F.conv1d(y, p[f"{prefix}.conv2.weight"], p[f"{prefix}.conv2.bias"]).transpose(-1, 1)

    def ln(self, prefix, x):
        return F.layer_norm(x, (x.shape[-1],), self.p[f"{prefix}.weight"], self.p[f"{prefix}.bias"], 1e-5)

    def conv_layer(self, prefix, x):
        """ConvLayer (encoder.py:22-28): circular conv → BatchNorm1d(eval) → ELU → MaxPool1d(3, 2, 1)."""
        p = self.p
        y = F.conv1d(F.pad(x.permute(0, 2, 1), (1, 1), mode="circular"), p[f"{prefix}.downConv.weight"],
                     p[f"{prefix}.downConv.bias"])
        y = F.batch_norm(y, p[f"{prefix}.norm.running_mean"], p[f"{prefix}.norm.running_var"],
                         p[f"{prefix}.norm.weight"], p[f"{prefix}.norm.bias"], False, 0.1, 1e-5)
        y = F.max_pool1d(F.elu(y), kernel_size=3, stride=2, padding=1)
        return y.transpose(1, 2)

    def encoder(self, prefix, n_layers, x, idx_iter, attns):
        """Encoder.forward (encoder.py:68-86)."""
        for l in range(n_layers):
            new_x, a = self.attention_layer(f"{prefix}.attn_layers.{l}.attention", x, x, self.cfg.attn, False, False,
                                            idx_iter, self.cfg.output_attention)
            lp = f"{prefix}.attn_layers.{l}"
            x = self.ln(f"{lp}.norm1", x + new_x)
            x = self.ln(f"{lp}.norm2", x + self.ffn(lp, x))
            attns.append(a)
            if self.cfg.distil and l < n_layers - 1:
                x = self.conv_layer(f"{prefix}.conv_layers.{l}", x)
        return self.ln(f"{prefix}.norm", x)

    @torch.no_grad()
    def forward(self, x_enc, x_dec, idx: Sequence[np.ndarray] = ()):
        """model.py:247-271 (InformerStack) / :115-139 (Informer) → ``out[B, pred_len, c_out]``."""
        cfg = self.cfg
        idx_iter = iter(list(idx))
        x = self.embed("enc_embedding", torch.as_tensor(x_enc).to(self.dt))
        attns = []
        if cfg.stack:                                                   # EncoderStack, encoder.py:95-106
            outs = []
            for i, el in enumerate(cfg.e_layers):
                inp_len = x.shape[1] // (2 ** i)
                outs.append(self.encoder(f"encoder.encoders.{i}", el, x[:, -inp_len:, :], idx_iter, attns))
            enc = torch.cat(outs, -2)
        else:
            enc = self.encoder("encoder", int(cfg.e_layers[0]), x, idx_iter, attns)
        d = self.embed("dec_embedding", torch.as_tensor(x_dec).to(self.dt))
        for l in range(cfg.d_layers):                                  # DecoderLayer, decoder.py:28-40
            lp = f"decoder.layers.{l}"
            sa, _ = self.attention_layer(f"{lp}.self_attention", d, d, cfg.attn, True, cfg.mix, idx_iter, False)
            d = self.ln(f"{lp}.norm1", d + sa)
            ca, _ = self.attention_layer(f"{lp}.cross_attention", d, enc, "full", False, False, idx_iter, False)
            d = self.ln(f"{lp}.norm2", d + ca)
            d = self.ln(f"{lp}.norm3", d + self.ffn(lp, d))
        d = self.ln("decoder.norm", d)
        y = F.linear(d, self.p["projection.weight"], self.p["projection.bias"])
        assert not list(idx_iter), "unused index samples"
        return y[:, -cfg.pred_len:, :]


def host_cpu() -> dict:
    """CPU model string and physical core count of this host (logical CPUs / threads per core)."""
    model, cores, sockets = "unknown", None, set()
    phys = set()
    try:
        with open("/proc/cpuinfo") as f:
            cur = {}
            for line in f:
                if not line.strip():
                    if "physical id" in cur and "core id" in cur:
                        phys.add((cur["physical id"], cur["core id"]))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name":
                    model = v.strip()
            if "physical id" in cur and "core id" in cur:
                phys.add((cur["physical id"], cur["core id"]))
        cores = len(phys) or None
    except OSError:
        pass
    import os

    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    return {"model": model, "physical_cores": cores, "usable_logical": usable}
