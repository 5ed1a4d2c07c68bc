"""GPU node-embedding index: the MI355X replacement of the reference's embedding matrix +
cosine/argsort top-k.

``VectorIndex`` wraps one ``hcr_index`` handle (one GPU, one row shard).  Semantics are the
reference's: sklearn cosine in fp64 over the stored rows, top-k ordered (score desc, row id
asc), optional ``(s+1)/2`` map and ``>= threshold`` filter (experiments/main.py:831-857,
experiments/isRelevant.py:197-210).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_float, c_int64, c_uint8, c_void_p

import numpy as np

from . import _lib
from ._lib import (HCR_BF16, HCR_F16, HCR_F32, HCR_SCORE_COSINE, HCR_SCORE_UNIT, SearchStats,
                   check, lib)

_DTYPES = {"f16": HCR_F16, "float16": HCR_F16, "bf16": HCR_BF16, "bfloat16": HCR_BF16,
           "f32": HCR_F32, "float32": HCR_F32}


def _np_rows(rows):
    """Host rows -> (contiguous array, hcr dtype).  float64 input is cast to float32."""
    a = np.asarray(rows)
    if a.dtype == np.float16:
        return np.ascontiguousarray(a), HCR_F16
    if a.dtype == np.uint16:          # raw bf16 bits
        return np.ascontiguousarray(a), HCR_BF16
    return np.ascontiguousarray(a, dtype=np.float32), HCR_F32


class VectorIndex:
    """Brute-force cosine top-k index on one MI355X.

    Parameters
    ----------
    dim : embedding width (384 MiniLM, 768 bge-base, 1024 bge-large, ...).
    dtype : storage dtype, "f16" (default), "bf16" or "f32".
    device : HIP device ordinal.
    capacity : rows to pre-reserve.
    """

    def __init__(self, dim: int, dtype: str = "f16", device: int = 0, capacity: int = 0):
        if dtype not in _DTYPES:
            raise ValueError(f"unknown dtype {dtype!r}")
        self._h = c_void_p()
        check(lib().hcr_index_create(int(device), int(dim), _DTYPES[dtype], int(capacity),
                                     ctypes.byref(self._h)))
        self.dim = int(dim)
        self.dtype = dtype
        self.device = int(device)
        self.id_offset = 0

    # -- lifecycle ----------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().hcr_index_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- contents -----------------------------------------------------------------------
    def __len__(self) -> int:
        return int(lib().hcr_index_size(self._h))

    def add(self, rows, normalize: bool = True) -> None:
        """Append rows (n x dim, float32/float64/float16, or uint16 bf16 bits)."""
        a, dt = _np_rows(rows)
        if a.ndim == 1:
            a = a.reshape(1, -1)
        if a.ndim != 2 or a.shape[1] != self.dim:
            raise ValueError(f"rows must be (n, {self.dim}), got {a.shape}")
        if a.shape[0] == 0:
            return
        check(lib().hcr_index_add(self._h, a.ctypes.data_as(c_void_p), int(a.shape[0]), dt,
                                  1 if normalize else 0))

    def add_ids(self, rows, ids, normalize: bool = True) -> None:
        """Append rows with explicit global ids (searches report these ids)."""
        a, dt = _np_rows(rows)
        if a.ndim == 1:
            a = a.reshape(1, -1)
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        if a.ndim != 2 or a.shape[1] != self.dim or ids.shape[0] != a.shape[0]:
            raise ValueError(f"rows must be (n, {self.dim}) with n ids")
        if a.shape[0] == 0:
            return
        check(lib().hcr_index_add_ids(self._h, a.ctypes.data_as(c_void_p), int(a.shape[0]), dt,
                                      1 if normalize else 0, ids.ctypes.data_as(c_void_p)))

    def add_device(self, ptr: int, n: int, rows_dtype: int, normalize: bool = False,
                   stream: int = 0) -> None:
        """Append n rows already in HBM (device pointer, e.g. ``tensor.data_ptr()``)."""
        check(lib().hcr_index_add_device(self._h, c_void_p(ptr), int(n), int(rows_dtype),
                                         1 if normalize else 0, c_void_p(stream or None)))

    def reset(self) -> None:
        """Drop all rows (device storage is kept for reuse)."""
        check(lib().hcr_index_reset(self._h))

    def set_id_offset(self, offset: int) -> None:
        check(lib().hcr_index_set_id_offset(self._h, int(offset)))
        self.id_offset = int(offset)

    def get_rows(self, row0: int = 0, n: int | None = None) -> np.ndarray:
        """Decoded stored rows as float32 (what the index actually ranks).  With
        ``normalize=True`` 16-bit rows are the input direction scaled to unit norm and rounded
        once -- the scale picked from 17 values within (1 +- 2^-9) of 1/||row|| so that the
        ROUNDED row's norm is closest to 1 (topk_kernels.h ingest_kernel) -- so they differ from
        a plain normalise-then-round of the input by a rounding step; cosine ranks are unchanged
        beyond the storage precision (tests/test_exact_gpu.py::test_normalized_16bit_store_ranks_
        like_the_inputs)."""
        if n is None:
            n = len(self) - row0
        out = np.empty((n, self.dim), dtype=np.float32)
        check(lib().hcr_index_get_rows(self._h, int(row0), int(n),
                                       out.ctypes.data_as(POINTER(c_float))))
        return out

    def set_rowmask(self, mask) -> None:
        """Restrict searches to rows with mask != 0 (None clears)."""
        if mask is None:
            check(lib().hcr_index_set_rowmask(self._h, None, 0))
            return
        m = np.ascontiguousarray(np.asarray(mask, dtype=bool).astype(np.uint8))
        check(lib().hcr_index_set_rowmask(self._h, m.ctypes.data_as(POINTER(c_uint8)),
                                          int(m.shape[0])))

    # -- queries ------------------------------------------------------------------------
    def search(self, queries, k: int, score_mode: int = HCR_SCORE_COSINE,
               threshold: float = -np.inf):
        """Exact top-k per query (any k >= 1; above 2048 by a sorted full scan).  Returns (scores float64 [nq,k] -- the exact
        fp64 cosine, mapped by ``score_mode`` --, ids int64 [nq,k]); -1 = empty slot."""
        q = np.ascontiguousarray(np.atleast_2d(np.asarray(queries, dtype=np.float32)))
        if q.shape[1] != self.dim:
            raise ValueError(
                f"Incompatible dimension for X and Y matrices: X.shape[1] == {q.shape[1]} "
                f"while Y.shape[1] == {self.dim}")
        nq = q.shape[0]
        s = np.empty((nq, k), dtype=np.float64)
        i = np.empty((nq, k), dtype=np.int64)
        check(lib().hcr_search(self._h, q.ctypes.data_as(POINTER(c_float)), nq, int(k),
                               int(score_mode), float(threshold),
                               s.ctypes.data_as(POINTER(c_double)),
                               i.ctypes.data_as(POINTER(c_int64))))
        return s, i

    def search_device(self, q_ptr: int, nq: int, k: int, out_scores_ptr: int, out_ids_ptr: int,
                      score_mode: int = HCR_SCORE_COSINE, threshold: float = -np.inf,
                      stream: int = 0) -> None:
        """HBM-resident variant: fp32 queries in, fp64 scores / int64 ids out (device ptrs)."""
        check(lib().hcr_search_device(self._h, c_void_p(q_ptr), int(nq), int(k),
                                      int(score_mode), float(threshold), c_void_p(out_scores_ptr),
                                      c_void_p(out_ids_ptr), c_void_p(stream or None)))

    def sample_device(self, q_ptr: int, nq: int, k: int, umax_ptr: int, umax_cap: int,
                      stream: int = 0):
        """Global seed, step 1 (hcr_search_sample_device): this shard's sampled unit maxima
        into umax_ptr ([units][nq] float32, umax_cap floats).  Returns (units, sampled_rows);
        units == 0: no sample on this shard's route."""
        u = ctypes.c_int(0)
        r = ctypes.c_int64(0)
        check(lib().hcr_search_sample_device(self._h, c_void_p(q_ptr), int(nq), int(k),
                                             c_void_p(umax_ptr), int(umax_cap), ctypes.byref(u),
                                             ctypes.byref(r), c_void_p(stream or None)))
        return u.value, r.value

    def search_seeded_device(self, q_ptr: int, nq: int, k: int, umax_all_ptr: int, units: int,
                             sampled_fraction: float, out_scores_ptr: int, out_ids_ptr: int,
                             out_bound_ptr: int, stream: int = 0) -> None:
        """Global seed, step 3 (hcr_search_seeded_device): this shard's exact top-k among the
        rows above the seed drawn from every shard's maxima, and per query the bound of the rest."""
        check(lib().hcr_search_seeded_device(self._h, c_void_p(q_ptr), int(nq), int(k),
                                             c_void_p(umax_all_ptr), int(units),
                                             float(sampled_fraction), c_void_p(out_scores_ptr),
                                             c_void_p(out_ids_ptr), c_void_p(out_bound_ptr),
                                             c_void_p(stream or None)))

    def score_all(self, queries, score_mode: int = HCR_SCORE_COSINE) -> np.ndarray:
        """Exact fp64 cosine of every (query, row): [nq, len(self)]."""
        q = np.ascontiguousarray(np.atleast_2d(np.asarray(queries, dtype=np.float32)))
        if q.shape[1] != self.dim:
            raise ValueError("dimension mismatch")
        out = np.empty((q.shape[0], len(self)), dtype=np.float64)
        check(lib().hcr_score_all(self._h, q.ctypes.data_as(POINTER(c_float)), q.shape[0],
                                  int(score_mode), out.ctypes.data_as(POINTER(c_double))))
        return out

    def last_stats(self) -> dict:
        st = SearchStats()
        check(lib().hcr_index_last_stats(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in SearchStats._fields_}

    def set_timing(self, enable: bool = True) -> None:
        """HIP-event timing of the fused score kernel (reported by ``last_stats``)."""
        check(lib().hcr_index_set_timing(self._h, 1 if enable else 0))

    OPT_QW1 = 1
    OPT_SAMPLE_STRIDE = 3
    OPT_QS_FORM = 4
    OPT_PREPASS = 5
    OPT_QW_DM = 6
    OPT_QW_MIN = 7
    OPT_QW_STAGGER = 8
    OPT_FLAG_READ = 9

    def set_option(self, option: int, value: int) -> None:
        """Kernel-choice option (``hcr_index_set_option``); never changes results.
        ``VectorIndex.OPT_QW1``: D = 1024 from 257 queries: -1 / 1 QW1 (default), 0 never (v4).
        ``VectorIndex.OPT_SAMPLE_STRIDE``: the sampling pre-pass's row-tile stride (0 heuristic).
        ``VectorIndex.OPT_QS_FORM``: QS ring stages at D = 384, 129-256 queries: 0 heuristic,
        1 64-deep, 3 128-deep.
        ``VectorIndex.OPT_PREPASS``: sampling pre-pass kernel, 1 v4, 2 QW (0 heuristic).
        ``VectorIndex.OPT_QW_DM``: QW's stage LDS-DMA issue, -1 default, 0 at the barrier, 3 spread.
        ``VectorIndex.OPT_QW_MIN``: smallest batch on the QW kernel (0 heuristic).
        ``VectorIndex.OPT_QW_STAGGER``: QW at D = 384, waves 4-7's test one stage late (-1 = 2, the default; 1 / 2 = two / one accumulator sets; 0 = off).
        ``VectorIndex.OPT_FLAG_READ``: the pass's certificate-count read back: 1 pageable copy, 2 pinned
        copy, 3 / 4 a kernel store into pinned host memory polled by the host (with / without a stream
        synchronisation after it); 0 the default."""
        check(lib().hcr_index_set_option(self._h, int(option), int(value)))

    TEST_PLANT_BAD_KEY = 1

    def test_hook(self, hook: int, value: int) -> None:
        """Per-handle test hook (``hcr_index_test_hook``; tests only, off by default)."""
        check(lib().hcr_index_test_hook(self._h, int(hook), int(value)))


class MultiDeviceIndex:
    """One process, several GPUs (``hcr_multi_*``): rows sharded in
    contiguous blocks over ``devices`` (a device may repeat), every shard searched concurrently,
    per-shard exact top-k lists gathered on ``devices[0]`` (RCCL sends over distinct devices,
    peer copies otherwise or when RCCL cannot create communicators) and merged there.  Same ``add`` / ``search`` /
    ``set_rowmask`` surface and results as ``VectorIndex`` over all rows."""

    def __init__(self, dim: int, devices, dtype: str = "f16", capacity: int = 0):
        if dtype not in _DTYPES:
            raise ValueError(f"unknown dtype {dtype!r}")
        devs = [int(d) for d in devices]
        if not devs:
            raise ValueError("need at least one device")
        arr = (ctypes.c_int * len(devs))(*devs)
        self._h = c_void_p()
        check(lib().hcr_multi_create(len(devs), arr, int(dim), _DTYPES[dtype], int(capacity),
                                     ctypes.byref(self._h)))
        self.dim = int(dim)
        self.dtype = dtype
        self.devices = devs

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().hcr_multi_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __len__(self) -> int:
        return int(lib().hcr_multi_size(self._h))

    def shard_sizes(self):
        return [int(lib().hcr_multi_shard_size(self._h, j)) for j in range(len(self.devices))]

    @property
    def exchange(self) -> str:
        """How the last search moved the per-shard lists: "rccl" or "peer"."""
        return {1: "rccl", 0: "peer"}.get(int(lib().hcr_multi_exchange_kind(self._h)), "?")

    def add(self, rows, normalize: bool = True) -> None:
        a, dt = _np_rows(rows)
        if a.ndim == 1:
            a = a.reshape(1, -1)
        if a.ndim != 2 or a.shape[1] != self.dim:
            raise ValueError(f"rows must be (n, {self.dim}), got {a.shape}")
        if a.shape[0] == 0:
            return
        check(lib().hcr_multi_add(self._h, a.ctypes.data_as(c_void_p), int(a.shape[0]), dt,
                                  1 if normalize else 0))

    def set_rowmask(self, mask) -> None:
        if mask is None:
            check(lib().hcr_multi_set_rowmask(self._h, None, 0))
            return
        m = np.ascontiguousarray(np.asarray(mask, dtype=bool).astype(np.uint8))
        check(lib().hcr_multi_set_rowmask(self._h, m.ctypes.data_as(POINTER(c_uint8)),
                                          int(m.shape[0])))

    def search(self, queries, k: int, score_mode: int = HCR_SCORE_COSINE,
               threshold: float = -np.inf):
        q = np.ascontiguousarray(np.atleast_2d(np.asarray(queries, dtype=np.float32)))
        if q.shape[1] != self.dim:
            raise ValueError(
                f"Incompatible dimension for X and Y matrices: X.shape[1] == {q.shape[1]} "
                f"while Y.shape[1] == {self.dim}")
        nq = q.shape[0]
        s = np.empty((nq, k), dtype=np.float64)
        i = np.empty((nq, k), dtype=np.int64)
        check(lib().hcr_multi_search(self._h, q.ctypes.data_as(POINTER(c_float)), nq, int(k),
                                     int(score_mode), float(threshold),
                                     s.ctypes.data_as(POINTER(c_double)),
                                     i.ctypes.data_as(POINTER(c_int64))))
        return s, i

    def last_stats(self) -> dict:
        st = SearchStats()
        check(lib().hcr_multi_last_stats(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in SearchStats._fields_}


def merge_topk_device(scores_ptr: int, ids_ptr: int, g: int, nq: int, k: int,
                      out_scores_ptr: int, out_ids_ptr: int, stream: int = 0) -> None:
    """Merge g shards' [g][nq][k] exact top-k lists on device."""
    check(lib().hcr_merge_topk_device(c_void_p(scores_ptr), c_void_p(ids_ptr), int(g), int(nq),
                                      int(k), c_void_p(out_scores_ptr), c_void_p(out_ids_ptr),
                                      c_void_p(stream or None)))


__all__ = ["VectorIndex", "MultiDeviceIndex", "merge_topk_device", "HCR_SCORE_COSINE", "HCR_SCORE_UNIT",
           "HCR_F16", "HCR_BF16", "HCR_F32", "_lib"]
