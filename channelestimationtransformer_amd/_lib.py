"""ctypes binding of the in-tree HIP engine library (``libcet.so``, C ABI of include/cet.h).

There is deliberately no fallback: if the library is missing or cannot be loaded the
import of this module fails with instructions to build it.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int64, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CET_LIB") or os.path.join(HERE, "libcet.so")   # CET_LIB: an A/B build


class CetError(RuntimeError):
    pass


class InformerConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("enc_in", "dec_in", "c_out", "seq_len", "label_len", "out_len", "factor",
                                     "d_model", "n_heads", "n_enc")] + [("e_layers", c_int * 4)] + \
               [(n, c_int) for n in ("d_layers", "d_ff", "attn_prob", "distil", "mix", "output_attention",
                                     "act_relu", "stack", "lsq_bits")]


class TransformerConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("src_vocab", "tgt_vocab", "src_seq_len", "tgt_seq_len", "label_len",
                                     "d_model", "N", "h", "d_ff")]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not found: build the HIP engine first "
                          f"(python -m channelestimationtransformer_amd.build)")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "cet_last_error": (c_char_p, []),
        "cet_version": (c_int, []),
        "cet_create_informer": (c_int, [POINTER(InformerConfig), POINTER(c_void_p)]),
        "cet_create_transformer": (c_int, [POINTER(TransformerConfig), POINTER(c_void_p)]),
        "cet_destroy": (None, [c_void_p]),
        "cet_load_weight": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
        "cet_missing_weights": (c_int, [c_void_p, c_char_p, c_int]),
        "cet_prob_calls": (c_int, [c_void_p, POINTER(c_int), c_int]),
        "cet_set_prob_indices": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int]),
        "cet_seed": (c_int, [c_void_p, c_uint64]),
        "cet_native_draw": (c_int64, [c_void_p, c_void_p, c_int64]),
        "cet_peek_draw": (c_int64, [c_void_p, c_void_p, c_int64]),
        "cet_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
        "cet_forward_nmse": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
        "cet_attns_floats": (c_int64, [c_void_p]),
        "cet_attns_layout": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int), c_int]),
        "cet_set_debug": (c_int, [c_void_p, c_void_p]),
        "cet_debug_floats": (c_int64, [c_void_p]),
        "cet_debug_layout": (c_int, [c_void_p, c_char_p, c_int]),
        "cet_nmse_split": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
        "cet_nmse_split_sums": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                                        c_void_p]),
        "cet_timing": (c_int, [c_void_p, c_int]),
        "cet_set_variant": (c_int, [c_void_p, c_int]),
        "cet_last_path": (c_int, [c_void_p]),
        "cet_last_kernel": (c_int, [c_void_p, c_char_p, c_int]),
        "cet_set_sampler": (c_int, [c_void_p, c_int]),
        "cet_set_precision": (c_int, [c_void_p, c_int]),
        "cet_get_precision": (c_int, [c_void_p]),
        "cet_set_stamps": (c_int, [c_void_p, c_void_p]),
        "cet_timing_read": (c_int, [c_void_p, POINTER(c_double), POINTER(c_int64)]),
        "cet_prepare_batch": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p,
                                      c_uint64, c_uint64, c_int, c_int, c_int, c_int, c_double, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p]),
        "cet_synth_channels": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_double,
                                       c_void_p, c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()
EXPORTED = ("cet_last_error", "cet_version", "cet_create_informer", "cet_create_transformer", "cet_destroy",
            "cet_load_weight", "cet_missing_weights", "cet_prob_calls", "cet_set_prob_indices", "cet_seed",
            "cet_native_draw", "cet_peek_draw",
            "cet_forward", "cet_forward_nmse", "cet_attns_floats", "cet_attns_layout", "cet_set_debug", "cet_debug_floats",
            "cet_debug_layout", "cet_nmse_split", "cet_nmse_split_sums", "cet_timing", "cet_timing_read",
            "cet_set_variant", "cet_last_path", "cet_last_kernel", "cet_set_sampler", "cet_set_precision", "cet_get_precision", "cet_set_stamps", "cet_prepare_batch", "cet_synth_channels")


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = lib.cet_last_error().decode(errors="replace")
        raise CetError(f"{what or 'cet'} failed ({rc}): {msg}")
    return rc
