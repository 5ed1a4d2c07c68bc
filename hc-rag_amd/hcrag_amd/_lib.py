"""ctypes binding of libhcrag_hip.so (C ABI declared in include/hcrag.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded,
``lib()`` raises.  (The CPU restatement under ``oracle/`` is test infrastructure only.)
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_uint8, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "HCRAG_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libhcrag_hip.so"))

HCR_OK, HCR_EINVAL, HCR_EHIP, HCR_ERCCL, HCR_ENOMEM, HCR_EIO, HCR_EINTERNAL = 0, -1, -2, -3, -4, -5, -6
HCR_F16, HCR_BF16, HCR_F32 = 0, 1, 2
HCR_SCORE_COSINE, HCR_SCORE_UNIT = 0, 1


class HcrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hcrag error {code}: {msg}")
        self.code = code


class SearchStats(ctypes.Structure):
    _fields_ = [("kprime", c_int32), ("widened_queries", c_int32),
                ("uncertified_queries", c_int32), ("partitions", c_int32),
                ("score_launches", c_int32), ("workgroups", c_int32),
                ("score_kernel_ms", c_double), ("unit_kernel", c_int32),
                ("fallback_queries", c_int32), ("fallback_rounds", c_int32),
                ("score_kernel", c_int32)]


class BertConfig(ctypes.Structure):
    """Mirror of ``hcr_bert_config`` (include/hcrag.h)."""
    _fields_ = [("vocab_size", c_int32), ("hidden", c_int32), ("layers", c_int32),
                ("heads", c_int32), ("intermediate", c_int32), ("max_position", c_int32),
                ("type_vocab", c_int32), ("layer_norm_eps", c_float), ("pooling", c_int32),
                ("normalize", c_int32)]


# name -> (restype, argtypes)
_SIGS = {
    "hcr_last_error": (c_char_p, []),
    "hcr_version": (c_char_p, []),
    "hcr_device_count": (c_int, []),
    "hcr_index_create": (c_int, [c_int, c_int, c_int, c_int64, POINTER(c_void_p)]),
    "hcr_index_destroy": (c_int, [c_void_p]),
    "hcr_index_reset": (c_int, [c_void_p]),
    "hcr_index_add": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int]),
    "hcr_index_add_device": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "hcr_index_set_id_offset": (c_int, [c_void_p, c_int64]),
    "hcr_index_add_ids": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "hcr_index_size": (c_int64, [c_void_p]),
    "hcr_index_dim": (c_int, [c_void_p]),
    "hcr_index_dtype": (c_int, [c_void_p]),
    "hcr_index_get_rows": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_float)]),
    "hcr_index_set_rowmask": (c_int, [c_void_p, POINTER(c_uint8), c_int64]),
    "hcr_search": (c_int, [c_void_p, POINTER(c_float), c_int64, c_int, c_int, c_double,
                           POINTER(c_double), POINTER(c_int64)]),
    "hcr_search_device": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int, c_double,
                                  c_void_p, c_void_p, c_void_p]),
    "hcr_search_sample_device": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64,
                                         POINTER(c_int), POINTER(c_int64), c_void_p]),
    "hcr_search_seeded_device": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int,
                                         c_double, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hcr_score_all": (c_int, [c_void_p, POINTER(c_float), c_int64, c_int, POINTER(c_double)]),
    "hcr_index_last_stats": (c_int, [c_void_p, POINTER(SearchStats)]),
    "hcr_index_set_timing": (c_int, [c_void_p, c_int]),
    "hcr_index_set_option": (c_int, [c_void_p, c_int, c_int]),
    "hcr_index_test_hook": (c_int, [c_void_p, c_int, c_int]),
    "hcr_merge_topk_device": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int, c_void_p,
                                      c_void_p, c_void_p]),
    "hcr_multi_create": (c_int, [c_int, POINTER(c_int), c_int, c_int, c_int64, POINTER(c_void_p)]),
    "hcr_multi_destroy": (c_int, [c_void_p]),
    "hcr_multi_add": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_int]),
    "hcr_multi_set_rowmask": (c_int, [c_void_p, POINTER(c_uint8), c_int64]),
    "hcr_multi_search": (c_int, [c_void_p, POINTER(c_float), c_int64, c_int, c_int, c_double,
                                 POINTER(c_double), POINTER(c_int64)]),
    "hcr_multi_size": (c_int64, [c_void_p]),
    "hcr_multi_num_shards": (c_int, [c_void_p]),
    "hcr_multi_shard_size": (c_int64, [c_void_p, c_int]),
    "hcr_multi_exchange_kind": (c_int, [c_void_p]),
    "hcr_multi_last_stats": (c_int, [c_void_p, POINTER(SearchStats)]),
    "hcr_wordpiece_create": (c_int, [c_char_p, c_int, c_int, POINTER(c_void_p)]),
    "hcr_wordpiece_create_from_buffer": (c_int, [c_char_p, c_int64, c_int, c_int,
                                                 POINTER(c_void_p)]),
    "hcr_wordpiece_destroy": (c_int, [c_void_p]),
    "hcr_wordpiece_vocab_size": (c_int32, [c_void_p]),
    "hcr_tokenize": (c_int, [c_void_p, POINTER(c_char_p), POINTER(c_int64), c_int64, c_int,
                             POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
    "hcr_encoder_create": (c_int, [c_int, POINTER(BertConfig), c_int, POINTER(c_void_p)]),
    "hcr_encoder_destroy": (c_int, [c_void_p]),
    "hcr_encoder_compute_dtype": (c_int, [c_void_p]),
    "hcr_encoder_set_weight": (c_int, [c_void_p, c_char_p, c_void_p, c_int64]),
    "hcr_encoder_finalize": (c_int, [c_void_p]),
    "hcr_encode": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "hcr_encode_device": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p,
                                  c_void_p]),
    "hcr_relevance_combine": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int, c_int64,
                                      c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                                      c_void_p]),
    "hcr_relevance_combine_device": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p,
                                             c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_int, c_void_p, c_int, c_void_p,
                                             c_void_p, c_void_p]),
}

_lib = None
_runtime = None


def _bind_hip_runtime():
    """One HIP runtime per process.

    PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7, but its libc10_hip
    NEEDs the file name ``libamdhip64.so``).  If /opt/rocm's runtime were loaded first (by
    this library) torch would load a second runtime and find no GPU.  So when torch is
    installed, preload torch's exact runtime files RTLD_GLOBAL: our NEEDED
    libamdhip64.so.7 then resolves to it by SONAME, and torch's later dlopen of the same
    file resolves to the same object.  ``HCRAG_HIP_RUNTIME=system`` skips this.
    """
    global _runtime
    if _runtime is not None or os.environ.get("HCRAG_HIP_RUNTIME") == "system":
        return
    import importlib.util
    _runtime = "system"
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    tl = os.path.join(os.path.dirname(spec.origin), "lib")
    hip = os.path.join(tl, "libamdhip64.so")
    if not os.path.exists(hip):
        return
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(tl, name)
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    _runtime = hip


def runtime_path() -> str:
    return _runtime or "unloaded"


def lib() -> ctypes.CDLL:
    """Load libhcrag_hip.so once (raises if it is missing: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libhcrag_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        _bind_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def declared_symbols():
    return list(_SIGS)


def check(rc: int) -> None:
    if rc != HCR_OK:
        msg = lib().hcr_last_error().decode("utf-8", "replace")
        if rc == HCR_EINVAL:
            raise ValueError(msg)
        raise HcrError(rc, msg)


def device_count() -> int:
    return int(lib().hcr_device_count())
