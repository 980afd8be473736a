"""nlp_amd -- MI355X-native neighborhood link prediction (host binding).

Python mirror of the reference's predict.hxx API over the C-ABI of
include/nlp.h (libnlp.so, HIP/gfx950).  The C++ mirror for main.cxx-style
callers is include/nlp/predict.hxx; this module serves the tests, bench.py and
the multi-GPU driver (dist.py).

Reference names (/root/reference/inc/predict.hxx):
    PredictLinkOptions{repeat, maxEdges, minScore}          predict.hxx:33-55
    PredictLinkResult{edges, time, scoringTime}             predict.hxx:65-102
    predictLinks<Metric>Omp<MINDEGREE1>(x, o)               predict.hxx:519-831
Here: predictLinks<Metric>Hip(graph, o, mindegree1=4) with the same meaning.

There is no CPU fallback: without libnlp.so or a gfx950 device every call
raises NlpError (the oracle under oracle/ is test infrastructure only).
"""
import ctypes
import operator
import os

import numpy as np

from . import build as _build

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NLP_LIB_PATH") or os.path.join(HERE, "libnlp.so")  # NLP_LIB_PATH: a variant build (experiments)

CN, JAC, SOR, SAL, HPI, HDI, LHN, AA, RA = range(9)
METRICS = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"]
METRIC_FUNCS = [
    "CommonNeighbors", "JaccardCoefficient", "SorensenIndex", "SaltonCosineSimilarity",
    "HubPromoted", "HubDepressed", "LeichtHolmeNermanScore", "AdamicAdarCoefficient",
    "ResourceAllocationScore",
]
STATUS = {0: "ok", 1: "invalid argument", 2: "HIP device error", 3: "out of memory",
          4: "no gfx950 device", 5: "output buffer too small"}
UINT64_MAX = (1 << 64) - 1

EDGE_DTYPE = np.dtype([("u", "<u4"), ("v", "<u4"), ("score", "<f4")])


class NlpError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__("%s: %s" % (what or "libnlp", STATUS.get(status, "status %d" % status)))


class Timing(ctypes.Structure):
    _fields_ = [("score_ms", ctypes.c_float), ("select_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
                ("copy_ms", ctypes.c_float), ("wedges", ctypes.c_uint64), ("candidates", ctypes.c_uint64),
                ("nan_candidates", ctypes.c_uint64), ("path", ctypes.c_uint32), ("chunks", ctypes.c_uint32),
                ("hot_ms", ctypes.c_float), ("graph_replay", ctypes.c_uint32), ("hot_bytes", ctypes.c_uint64),
                ("hot_kernel", ctypes.c_uint32), ("call_bytes", ctypes.c_uint64), ("order_route", ctypes.c_uint32)]

    def as_dict(self):
        return dict(zip(_TIMING_FIELDS, _timing_get(self)))


_TIMING_FIELDS = tuple(f for f, _ in Timing._fields_)
_timing_get = operator.attrgetter(*_TIMING_FIELDS)

EXPORTS = [
    "nlp_graph_create", "nlp_graph_create_device", "nlp_graph_destroy", "nlp_graph_info", "nlp_predict",
    "nlp_predict_ex", "nlp_copy_last", "nlp_predict_device", "nlp_predict_device_ex", "nlp_predict_device_async",
    "nlp_sync", "nlp_select_edges_device",
    "nlp_merge_blocks_device", "nlp_set_truth", "nlp_count_common_device", "nlp_last_common", "nlp_status_string",
    "nlp_metric_name", "nlp_version", "nlp_graph_create_multi", "nlp_device_count", "nlp_graph_parts",
    "nlp_ingest_device", "nlp_delete_edges_device", "nlp_host_alloc", "nlp_host_free", "nlp_graph_build_phases",
    "nlp_set_hot_stage",
]

_lib = None


def lib(build_if_missing=True):
    """Load libnlp.so (building it first when it is missing and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH) and build_if_missing:
        _build.build()
    if not os.path.exists(LIB_PATH):
        raise NlpError(4, "libnlp.so missing (run neighborhood-link-prediction-openmp_amd/build.py)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, f32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, ctypes.c_int
    P = ctypes.POINTER
    L.nlp_graph_create.argtypes = [vp, vp, u64, i32, P(vp)]
    L.nlp_graph_create_device.argtypes = [vp, vp, u64, u64, i32, vp, P(vp)]
    L.nlp_graph_create_multi.argtypes = [vp, vp, u64, vp, i32, P(vp)]
    L.nlp_graph_create_multi.restype = i32
    L.nlp_device_count.restype = i32
    L.nlp_graph_parts.argtypes = [vp, P(i32), vp]
    L.nlp_graph_parts.restype = i32
    L.nlp_ingest_device.argtypes = [vp, vp, u64, u64, i32, vp, vp, u64, P(u64), i32, vp]
    L.nlp_ingest_device.restype = i32
    L.nlp_delete_edges_device.argtypes = [vp, vp, u64, u64, P(u32), vp, vp, P(u64), vp, vp, P(u64), i32, vp]
    L.nlp_delete_edges_device.restype = i32
    L.nlp_graph_destroy.argtypes = [vp]
    L.nlp_graph_destroy.restype = None
    L.nlp_graph_info.argtypes = [vp, P(u64), P(u64), P(u32), P(i32)]
    L.nlp_graph_build_phases.argtypes = [vp, u32, P(u32), vp, vp, P(ctypes.c_double)]
    L.nlp_graph_build_phases.restype = i32
    L.nlp_set_hot_stage.argtypes = [vp, i32]
    L.nlp_set_hot_stage.restype = i32
    L.nlp_predict.argtypes = [vp, i32, u32, f32, u64, i32, vp, P(u64), P(Timing)]
    L.nlp_predict_ex.argtypes = [vp, i32, u32, u32, f32, u64, i32, vp, P(u64), P(Timing)]
    L.nlp_copy_last.argtypes = [vp, vp, u64, P(u64)]
    L.nlp_predict_device.argtypes = [vp, i32, u32, f32, u64, u64, u64, vp, P(u64), P(Timing), vp]
    L.nlp_predict_device_ex.argtypes = [vp, i32, u32, u32, f32, u64, u64, u64, vp, P(u64), P(Timing), vp]
    L.nlp_predict_device_async.argtypes = [vp, i32, u32, u32, f32, u64, u64, u64, vp, vp]
    L.nlp_sync.argtypes = [vp, P(u64), P(Timing)]
    L.nlp_select_edges_device.argtypes = [vp, vp, u64, u64, vp, P(u64), vp]
    L.nlp_merge_blocks_device.argtypes = [vp, vp, u64, u32, u64, vp, P(u64), vp]
    L.nlp_set_truth.argtypes = [vp, vp, vp, u64]
    L.nlp_count_common_device.argtypes = [vp, vp, u64, P(u64), vp]
    L.nlp_last_common.argtypes = [vp, P(u64)]
    L.nlp_status_string.argtypes = [i32]
    L.nlp_status_string.restype = ctypes.c_char_p
    L.nlp_metric_name.argtypes = [i32]
    L.nlp_metric_name.restype = ctypes.c_char_p
    L.nlp_version.restype = i32
    for f in ("nlp_graph_create", "nlp_graph_create_device", "nlp_graph_info", "nlp_predict", "nlp_predict_ex",
              "nlp_copy_last", "nlp_predict_device", "nlp_predict_device_ex", "nlp_predict_device_async", "nlp_sync",
              "nlp_select_edges_device",
              "nlp_merge_blocks_device", "nlp_set_truth", "nlp_count_common_device", "nlp_last_common"):
        getattr(L, f).restype = i32
    _lib = L
    return L


def _check(status, what):
    if status != 0:
        raise NlpError(status, what)


def _metric(m):
    if isinstance(m, str):
        return METRICS.index(m)
    if not 0 <= int(m) <= 8:
        raise ValueError("metric out of range")
    return int(m)


def _check_tensor(t, name, dtypes, device=None, min_numel=0):
    """Raise ValueError unless `t` is a contiguous torch tensor of one of
    `dtypes` on the GPU (`device`: the graph's ordinal) with >= min_numel
    elements: the library gets t.data_ptr() and trusts its layout."""
    import torch
    if not isinstance(t, torch.Tensor):
        raise ValueError("%s must be a torch tensor" % name)
    if t.dtype not in dtypes:
        raise ValueError("%s must have dtype %s, got %s" % (name, "/".join(str(d) for d in dtypes), t.dtype))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)
    if not t.is_cuda or (device is not None and t.device.index != device):
        raise ValueError("%s must live on cuda:%s, got %s" % (name, device, t.device))
    if t.numel() < min_numel:
        raise ValueError("%s too small: %d elements, need %d" % (name, t.numel(), min_numel))


_EDGE_DTYPES = None


def _edge_dtypes():
    global _EDGE_DTYPES
    if _EDGE_DTYPES is None:
        import torch
        _EDGE_DTYPES = (torch.int32, torch.uint32) if hasattr(torch, "uint32") else (torch.int32,)
    return _EDGE_DTYPES


def _stream_ptr(stream, tensor=None):
    """hipStream_t for the library: the given stream, else torch's current
    stream when the operands are torch device tensors (so that library kernels
    are ordered after the kernels that produced them)."""
    if stream is None and tensor is not None and getattr(tensor, "is_cuda", False):
        import torch
        stream = torch.cuda.current_stream(tensor.device)
    if stream is None:
        return None
    return getattr(stream, "cuda_stream", stream)


class PredictLinkOptions:
    """predict.hxx:33-55: repeat [1], maxEdges [-1 = all], minScore [0]."""

    def __init__(self, repeat=1, maxEdges=-1, minScore=0.0):
        self.repeat = int(repeat)
        self.maxEdges = int(maxEdges)
        self.minScore = float(minScore)


class PredictLinkResult:
    """predict.hxx:65-102: edges [(u, v, score)] by score desc, time / scoringTime in ms."""

    def __init__(self, edges, time=0.0, scoringTime=0.0, timing=None):
        self.edges = edges
        self.time = time
        self.scoringTime = scoringTime
        self.timing = timing or {}


class Graph:
    """A CSR graph resident in HBM (nlp_graph handle).

    offsets: u64[span+1], keys: u32[nnz]; rows sorted ascending, duplicates
    allowed (the reference's LazyBitset multiset semantics)."""

    def __init__(self, offsets, keys, device=0, devices=None):
        """devices: a list of HIP ordinals, one per source partition (repeats =
        logical partitions on one device) -> nlp_graph_create_multi; results
        are identical to a single-device graph and device outputs live on
        devices[0]."""
        L = lib()
        self._off = np.ascontiguousarray(offsets, dtype=np.uint64)
        self._keys = np.ascontiguousarray(keys, dtype=np.uint32)
        span = len(self._off) - 1
        h = ctypes.c_void_p()
        kp = self._keys.ctypes.data if len(self._keys) else None
        if devices is not None:
            devs = np.ascontiguousarray(np.asarray(devices, dtype=np.int32))
            _check(L.nlp_graph_create_multi(self._off.ctypes.data, kp, span, devs.ctypes.data, len(devs),
                                            ctypes.byref(h)), "nlp_graph_create_multi")
            device = int(devs[0]) if len(devs) else 0
        else:
            _check(L.nlp_graph_create(self._off.ctypes.data, kp, span, int(device), ctypes.byref(h)),
                   "nlp_graph_create")
        self._h = h
        self.device = int(device)
        del self._off, self._keys

    def parts(self):
        """(number of partitions, their source bounds of the last prediction or None)."""
        L = lib()
        n = ctypes.c_int()
        _check(L.nlp_graph_parts(self._h, ctypes.byref(n), None), "nlp_graph_parts")
        b = np.zeros(n.value + 1, np.uint64)
        st = L.nlp_graph_parts(self._h, ctypes.byref(n), b.ctypes.data)
        return n.value, (b if st == 0 else None)

    @classmethod
    def from_device(cls, offsets, keys, device=None, stream=None):
        """From torch tensors already on the GPU (int64 offsets, int32 keys)."""
        import torch
        L = lib()
        g = cls.__new__(cls)
        dev = offsets.device.index if device is None else device
        _check_tensor(offsets, "offsets", (torch.int64,) + ((torch.uint64,) if hasattr(torch, "uint64") else ()),
                      dev, 1)
        _check_tensor(keys, "keys", (torch.int32,) + ((torch.uint32,) if hasattr(torch, "uint32") else ()), dev)
        span = offsets.numel() - 1
        h = ctypes.c_void_p()
        _check(L.nlp_graph_create_device(offsets.data_ptr(), keys.data_ptr() if keys.numel() else None, span,
                                         keys.numel(), int(dev or 0), _stream_ptr(stream, offsets), ctypes.byref(h)),
               "nlp_graph_create_device")
        g._h = h
        g.device = int(dev or 0)
        return g

    def info(self):
        s, m, d, y = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_int()
        _check(lib().nlp_graph_info(self._h, ctypes.byref(s), ctypes.byref(m), ctypes.byref(d), ctypes.byref(y)),
               "nlp_graph_info")
        return dict(span=s.value, nnz=m.value, max_degree=d.value, symmetric=bool(y.value))

    def set_hot_stage(self, stage):
        """nlp_set_hot_stage: time sort-path stage `stage` with HIP events (-1: the kernels' stamps)."""
        _check(lib().nlp_set_hot_stage(self._h, int(stage)), "nlp_set_hot_stage")

    def build_phases(self):
        """Where the create call's time went (nlp_graph_build_phases): an
        ordered {phase: ms} dict (host wall time, the stream drained at each
        phase boundary) plus 'hipMalloc_ms', the part spent inside hipMalloc."""
        L = lib()
        n = ctypes.c_uint32()
        names = (ctypes.c_char_p * 32)()
        ms = (ctypes.c_double * 32)()
        alloc = ctypes.c_double()
        _check(L.nlp_graph_build_phases(self._h, 32, ctypes.byref(n), names, ms, ctypes.byref(alloc)),
               "nlp_graph_build_phases")
        out = {names[i].decode(): ms[i] for i in range(min(n.value, 32))}
        out["hipMalloc_ms"] = alloc.value
        return out

    def predict(self, metric, hub, max_edges=None, min_score=0.0, repeat=1, maxfactor2=0):
        """Host-output predict: returns (u, v, score) numpy arrays and the timing dict.
        maxfactor2: the reference's MAXFACTOR2 template parameter (0 = off)."""
        L = lib()
        m = _metric(metric)
        me = UINT64_MAX if max_edges is None or max_edges < 0 else int(max_edges)
        t = Timing()
        cnt = ctypes.c_uint64()
        if me == UINT64_MAX:
            # all candidates: one prediction kept on the device (out = NULL), then fetched
            _check(L.nlp_predict_ex(self._h, m, int(hub), int(maxfactor2), float(min_score), me, int(repeat), None,
                                    ctypes.byref(cnt), ctypes.byref(t)), "nlp_predict_ex")
            out = np.zeros(max(cnt.value, 1), dtype=EDGE_DTYPE)
            got = ctypes.c_uint64()
            _check(L.nlp_copy_last(self._h, out.ctypes.data, cnt.value, ctypes.byref(got)), "nlp_copy_last")
            n = got.value
        else:
            out = np.zeros(max(me, 1), dtype=EDGE_DTYPE)
            _check(L.nlp_predict_ex(self._h, m, int(hub), int(maxfactor2), float(min_score), me, int(repeat),
                                    out.ctypes.data if me else None, ctypes.byref(cnt), ctypes.byref(t)),
                   "nlp_predict_ex")
            n = cnt.value
        out = out[:n]
        return out["u"].copy(), out["v"].copy(), out["score"].copy(), t.as_dict()

    def predict_device(self, metric, hub, max_edges, out, u_begin=0, u_end=UINT64_MAX, min_score=0.0, stream=None,
                       maxfactor2=0):
        """Device-output predict into `out` (torch int32 [>= max_edges, 3]).  Returns (count, timing)."""
        # the per-call Python is part of every step: the output tensor's checks
        # are remembered for the same tensor and size, the result structs reused
        need = 3 * int(max_edges)
        memo = (id(out), out.data_ptr(), need, out.dtype, out.is_contiguous(), out.numel())
        if getattr(self, "_out_ok", None) != memo:
            _check_tensor(out, "out", _edge_dtypes(), self.device, need)
            self._out_ok = memo
        io = getattr(self, "_io", None)
        if io is None:
            t, cnt = Timing(), ctypes.c_uint64()
            io = self._io = (t, cnt, ctypes.byref(cnt), ctypes.byref(t), lib().nlp_predict_device_ex)
        t, cnt, rcnt, rt, fn = io
        _check(fn(self._h, _metric(metric), int(hub), int(maxfactor2), float(min_score), int(max_edges), int(u_begin),
                  int(u_end), out.data_ptr(), rcnt, rt, _stream_ptr(stream, out)), "nlp_predict_device_ex")
        return cnt.value, t.as_dict()

    def predict_device_async(self, metric, hub, max_edges, out, u_begin=0, u_end=UINT64_MAX, min_score=0.0,
                             stream=None, maxfactor2=0):
        """nlp_predict_device_async: enqueue predict_device's computation without a
        host wait (it runs synchronously unless the same call last ran
        synchronously as one replayed graph); results after sync()."""
        need = 3 * int(max_edges)
        memo = (id(out), out.data_ptr(), need, out.dtype, out.is_contiguous(), out.numel())
        if getattr(self, "_out_ok", None) != memo:
            _check_tensor(out, "out", _edge_dtypes(), self.device, need)
            self._out_ok = memo
        fn = getattr(self, "_afn", None) or lib().nlp_predict_device_async
        self._afn = fn
        _check(fn(self._h, _metric(metric), int(hub), int(maxfactor2), float(min_score), int(max_edges), int(u_begin),
                  int(u_end), out.data_ptr(), _stream_ptr(stream, out)), "nlp_predict_device_async")

    def sync(self):
        """nlp_sync: wait for the predict_device_async batch; (count, timing) of its
        last call.  NlpError(NLP_ERR_RETRY = 6) when a call of the batch needs a
        synchronous redo."""
        t, cnt = Timing(), ctypes.c_uint64()
        _check(lib().nlp_sync(self._h, ctypes.byref(cnt), ctypes.byref(t)), "nlp_sync")
        return cnt.value, t.as_dict()

    def select_edges_device(self, edges_in, n, max_edges, out, stream=None):
        _check_tensor(edges_in, "edges_in", _edge_dtypes(), self.device, 3 * int(n))
        _check_tensor(out, "out", _edge_dtypes(), self.device, 3 * min(int(n), int(max_edges)))
        cnt = ctypes.c_uint64()
        _check(lib().nlp_select_edges_device(self._h, edges_in.data_ptr(), int(n), int(max_edges), out.data_ptr(),
                                             ctypes.byref(cnt), _stream_ptr(stream, out)), "nlp_select_edges_device")
        return cnt.value

    def merge_blocks_device(self, blocks, max_edges, out, stream=None):
        """Merge the gathered shard blocks (torch int32 [nblocks, stride, 3], entry 0
        of each block a header, nlp.h nlp_merge_blocks_device) into `out`.  Returns
        the merged count, or raises NlpError(NLP_ERR_CAPACITY) with .count = the
        largest block count when a block overflowed its stride."""
        _check_tensor(blocks, "blocks", _edge_dtypes(), self.device)
        if blocks.dim() != 3 or blocks.shape[2] != 3:
            raise ValueError("blocks must be [nblocks, stride, 3]")
        _check_tensor(out, "out", _edge_dtypes(), self.device,
                      3 * min(int(max_edges), int(blocks.shape[0]) * int(blocks.shape[1])))
        cnt = ctypes.c_uint64()
        st = lib().nlp_merge_blocks_device(self._h, blocks.data_ptr(), int(blocks.shape[1]), int(blocks.shape[0]),
                                           int(max_edges), out.data_ptr(), ctypes.byref(cnt), _stream_ptr(stream, out))
        if st == 5:
            e = NlpError(st, "nlp_merge_blocks_device")
            e.count = cnt.value
            raise e
        _check(st, "nlp_merge_blocks_device")
        return cnt.value

    def set_truth(self, del_u, del_w):
        """Directed deletions (main.cxx deletions0) for the device evaluation."""
        u = np.ascontiguousarray(np.asarray(del_u, dtype=np.uint32))
        w = np.ascontiguousarray(np.asarray(del_w, dtype=np.uint32))
        _check(lib().nlp_set_truth(self._h, u.ctypes.data, w.ctypes.data, len(u)), "nlp_set_truth")

    def count_common_device(self, edges, n, stream=None):
        """|insertions1 ∩ deletions0| for the first n device edges (torch int32 [>= n, 3])."""
        _check_tensor(edges, "edges", _edge_dtypes(), self.device, 3 * int(n))
        c = ctypes.c_uint64()
        _check(lib().nlp_count_common_device(self._h, edges.data_ptr(), int(n), ctypes.byref(c),
                                             _stream_ptr(stream, edges)), "nlp_count_common_device")
        return c.value

    def last_common(self):
        c = ctypes.c_uint64()
        _check(lib().nlp_last_common(self._h, ctypes.byref(c)), "nlp_last_common")
        return c.value

    def close(self):
        if getattr(self, "_h", None):
            lib().nlp_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def ingest_device(src, dst, n, symmetric_input=False, stream=None):
    """SURVEY §8(f) N1 on the device (nlp_ingest_device): the reference's
    readMtx rows, symmetrize (duplicate rule included) and self-loop removal
    from the file's directed pairs (torch int32 device tensors, 1-based ids
    <= n).  Returns (offsets int64 [n + 2], keys int32 [nnz]) on the device."""
    import torch
    dev = src.device.index or 0
    _check_tensor(src, "src", (torch.int32,), dev)
    _check_tensor(dst, "dst", (torch.int32,), dev, src.numel())
    m = src.numel()
    off = torch.empty(n + 2, dtype=torch.int64, device=src.device)
    keys = torch.empty(max(2 * m, 1), dtype=torch.int32, device=src.device)
    nnz = ctypes.c_uint64()
    _check(lib().nlp_ingest_device(src.data_ptr() if m else None, dst.data_ptr() if m else None, m, int(n),
                                   int(bool(symmetric_input)), off.data_ptr(), keys.data_ptr(), keys.numel(),
                                   ctypes.byref(nnz), dev, _stream_ptr(stream, src)), "nlp_ingest_device")
    return off, keys[:nnz.value].clone()


def delete_edges_device(offsets, keys, batch, rng_state, stream=None):
    """SURVEY §8(f) N2 on the device (nlp_delete_edges_device): one deletion
    batch drawn by std::default_random_engine at `rng_state` (the seed of a
    fresh engine, or the state a previous call returned), tidied and applied.
    Returns (offsets', keys', del_u, del_v, rng_state') -- the deletions
    directed, sorted, unique (main.cxx deletions0)."""
    import torch
    dev = offsets.device.index or 0
    _check_tensor(offsets, "offsets", (torch.int64,), dev, 1)
    _check_tensor(keys, "keys", (torch.int32,), dev)
    span = offsets.numel() - 1
    off2 = torch.empty_like(offsets)
    keys2 = torch.empty(max(keys.numel(), 1), dtype=torch.int32, device=keys.device)
    du = torch.empty(max(2 * int(batch), 1), dtype=torch.int32, device=keys.device)
    dv = torch.empty_like(du)
    st = ctypes.c_uint32(int(rng_state) & 0xFFFFFFFF)
    n2, nd = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().nlp_delete_edges_device(offsets.data_ptr(), keys.data_ptr() if keys.numel() else None, span,
                                         int(batch), ctypes.byref(st), off2.data_ptr(), keys2.data_ptr(),
                                         ctypes.byref(n2), du.data_ptr(), dv.data_ptr(), ctypes.byref(nd), dev,
                                         _stream_ptr(stream, offsets)), "nlp_delete_edges_device")
    return off2, keys2[:n2.value].clone(), du[:nd.value].clone(), dv[:nd.value].clone(), st.value


def _make_predictor(metric):
    def fn(x, o=None, mindegree1=4, maxfactor2=0):
        o = o or PredictLinkOptions()
        u, v, s, t = x.predict(metric, mindegree1, None if o.maxEdges < 0 else o.maxEdges, o.minScore, o.repeat,
                               maxfactor2)
        edges = list(zip(u.tolist(), v.tolist(), s.tolist()))
        return PredictLinkResult(edges, t["total_ms"], t["score_ms"], t)
    fn.__name__ = "predictLinks%sHip" % METRIC_FUNCS[metric]
    fn.__doc__ = ("predictLinks%sOmp<MINDEGREE1, MAXFACTOR2>(x, o) of predict.hxx on the GPU "
                  "(mindegree1=0 -> IHub, maxfactor2=0 -> off)." % METRIC_FUNCS[metric])
    return fn


for _m, _name in enumerate(METRIC_FUNCS):
    globals()["predictLinks%sHip" % _name] = _make_predictor(_m)
del _m, _name


def edges_from_tensor(t, n):
    """Split a device edge tensor (int32 [cap, 3]) into numpy u, v, score."""
    a = t[:n].cpu().numpy()
    return a[:, 0].view(np.uint32).copy(), a[:, 1].view(np.uint32).copy(), a[:, 2].view(np.float32).copy()
