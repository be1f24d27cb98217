"""ctypes binding of include/fastbn.h and the reference-shaped Python classes."""
import atexit
import ctypes as C
import weakref
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FBN_LIB_PATH: an alternative build of the same library (A/B runs of build-time switches, tools/)
LIB_PATH = os.environ.get("FBN_LIB_PATH") or os.path.join(_HERE, "libfastbn.so")

_vp, _i32, _i64, _dbl, _cstr = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_char_p
_pp = C.POINTER(C.c_void_p)

# name -> argtypes (all functions return int status except fbn_last_error)
_SIGS = {
    "fbn_version": [_vp, _vp],
    "fbn_device_count": [_vp],
    "fbn_network_load_xmlbif": [_cstr, _pp],
    "fbn_network_create": [C.c_int, _vp, _vp, _vp, _vp, _vp, _pp],
    "fbn_network_node_counts": [_vp, C.c_int, _vp, _vp, _vp, _vp],
    "fbn_network_num_nodes": [_vp, _vp],
    "fbn_network_dims": [_vp, _vp],
    "fbn_network_name": [_vp, C.c_int, C.c_char_p, C.c_int],
    "fbn_network_destroy": [_vp],
    "fbn_evidence_load_libsvm": [_cstr, C.c_int, _vp, _vp, _i64, _vp],
    "fbn_dataset_load_csv": [_cstr, _pp],
    "fbn_synth_forward_sample": [_vp, _i64, C.c_uint64, _vp],
    "fbn_synth_evidence": [_vp, _i64, C.c_int, C.c_uint64, C.c_int, _vp],
    "fbn_write_csv": [_cstr, _vp, C.c_int, _i64, _vp],
    "fbn_write_libsvm": [_cstr, _vp, _i64, C.c_int, _vp],
    "fbn_dataset_shape": [_vp, _vp, _vp],
    "fbn_dataset_dims": [_vp, _vp],
    "fbn_dataset_columns": [_vp, _vp],
    "fbn_dataset_var_name": [_vp, C.c_int, C.c_char_p, C.c_int],
    "fbn_dataset_destroy": [_vp],
    "fbn_jt_plan_create": [_vp, C.c_int, _pp],
    "fbn_jt_plan_info_get": [_vp, _vp],
    "fbn_jt_plan_dump": [_vp, _cstr, _cstr],
    "fbn_jt_run": [_vp, _vp, _i64, _vp, _vp, _vp],
    "fbn_jt_run_device": [_vp, _vp, _i64, _vp, _vp, _vp],
    "fbn_jt_evidence_validate": [_vp, _vp, _i64, _vp],
    "fbn_jt_set_evidence_check": [_vp, C.c_int],
    "fbn_jt_set_kernel_timing": [_vp, C.c_int],
    "fbn_jt_score": [_vp, _vp, _vp, _i64, _vp, _vp],
    "fbn_jt_set_output_layout": [_vp, C.c_int],
    "fbn_jt_score_terms_device": [_vp, _vp, _vp, _i64, _vp, _vp],
    "fbn_jt_last_kernel_ms": [_vp, _vp],
    "fbn_jt_stream_schedule": [_vp, _vp, C.c_int64, _vp, C.c_int64, _vp, _vp],
    "fbn_jt_set_waves_per_cu": [_vp, C.c_int],
    "fbn_jt_set_variant": [_vp, C.c_int],
    "fbn_jt_debug_op_cycles": [_vp, C.c_int, _vp],
    "fbn_jt_kernel_source": [_vp, C.c_char_p, C.c_int64, _vp],
    "fbn_jt_kernel_cache_path": [_vp, C.c_char_p, C.c_int64],
    "fbn_jt_kernel_options": [C.c_char_p, C.c_int64],
    "fbn_jt_kernel_build": [_vp],
    "fbn_jt_debug_force_fixup": [_vp, C.c_int],
    "fbn_jt_debug_flagged_blocks": [_vp, _vp],
    "fbn_jt_set_exact": [_vp, C.c_int],
    "fbn_jt_plan_destroy": [_vp],
    "fbn_ci_dataset_upload": [_vp, C.c_int, _i64, _vp, C.c_int, _pp],
    "fbn_ci_dataset_from_device": [_vp, C.c_int, _i64, _vp, C.c_int, _pp],
    "fbn_ci_set_kernel_timing": [_vp, C.c_int],
    "fbn_ci_run": [_vp, _vp, _i64, C.c_int, _dbl, _vp, _vp, _vp, _vp, _vp],
    "fbn_ci_counts": [_vp, C.c_int, C.c_int, _vp, C.c_int, _vp, _i64, _vp],
    "fbn_ci_last_kernel_ms": [_vp, _vp],
    "fbn_ci_decision_margin": [_vp, _vp, _vp, C.c_int],
    "fbn_ci_debug_counts": [_vp, _vp, _i64, C.c_int, _vp, _i64],
    "fbn_pc_decision_margin": [_vp, _vp, _vp],
    "fbn_ci_ctx_destroy": [_vp],
    "fbn_pc_stable": [_vp, _dbl, C.c_int, C.c_int, _pp],
    "fbn_pc_num_levels": [_vp, _vp],
    "fbn_pc_level_tests": [_vp, _vp],
    "fbn_pc_level_launched": [_vp, _vp],
    "fbn_pc_num_edges": [_vp, _vp],
    "fbn_pc_edges": [_vp, _vp],
    "fbn_pc_sepsets": [_vp, _vp, _i64, _vp],
    "fbn_pc_timing": [_vp, _vp, _vp],
    "fbn_pc_path": [_vp, _vp],
    "fbn_jt_tile_program": [_vp, _vp, _vp, _vp, _vp],
    "fbn_pc_result_record": [_vp, _vp, C.c_int64, _vp],
    "fbn_pc_small_eligible": [_vp, C.c_int, _vp],
    "fbn_pc_small_eligible_shape": [C.c_int, C.c_int64, _vp, C.c_int, _vp],
    "fbn_pc_device_bytes": [_vp, _vp],
    "fbn_pc_orient_skeleton": [C.c_int, _vp, C.c_int, _vp, C.c_int64, _vp],
    "fbn_pc_level": [_vp, C.c_double, C.c_int, C.c_int, _vp, C.c_int64, C.c_int64, C.c_int64, _vp, _vp, _vp, _vp],
    "fbn_pc_num_oriented_edges": [_vp, _vp],
    "fbn_pc_oriented_edges": [_vp, _vp],
    "fbn_pc_shd_bif": [_vp, C.c_char_p, _vp],
    "fbn_shd_bif": [C.c_char_p, C.c_int, _vp, C.c_int, _vp],
    "fbn_pc_result_destroy": [_vp],
    "fbn_pc_dist_create": [C.c_int, _dbl, C.c_int, C.c_int, _pp],
    "fbn_pc_dist_level": [_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp],
    "fbn_pc_dist_num_edges": [_vp, _vp],
    "fbn_pc_dist_edges": [_vp, _vp, _i64],
    "fbn_pc_dist_run": [_vp, _vp, _vp],
    "fbn_pc_dist_pack": [_vp, _vp, _vp, _i64, _i64, _vp],
    "fbn_pc_dist_pairs_chunk": [_vp, _vp],
    "fbn_pc_dist_pairs_export": [_vp, _vp, C.c_int],
    "fbn_pc_dist_pairs_import": [_vp, _vp, _vp, C.c_int],
    "fbn_pc_dist_apply": [_vp, _vp, _vp],
    "fbn_pc_dist_result": [_vp, _pp],
    "fbn_pc_dist_destroy": [_vp],
}


class FastBNError(RuntimeError):
    pass


class _Lib:
    """Lazily loaded libfastbn.so.  Missing library => every call raises (no CPU fallback)."""

    def __init__(self):
        self._h = None

    def load(self):
        if self._h is None:
            if not os.path.exists(LIB_PATH):
                raise FastBNError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback)")
            try:
                # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's): load it first
                # so that one HIP runtime serves both when they share a process
                import torch  # noqa: F401
            except ImportError:
                pass
            h = C.CDLL(LIB_PATH)
            for name, args in _SIGS.items():
                f = getattr(h, name)
                f.argtypes = args
                f.restype = C.c_int
            h.fbn_last_error.restype = C.c_char_p
            h.fbn_last_error.argtypes = []
            self._h = h
        return self._h

    def __getattr__(self, name):
        h = self.load()
        f = getattr(h, name)
        if name == "fbn_last_error":
            return f

        def call(*args):
            rc = f(*args)
            if rc != 0:
                raise FastBNError(f"{name}: {h.fbn_last_error().decode()} (code {rc})")
            return rc

        return call


lib = _Lib()

# Every live handle (networks, datasets, plans, CI contexts, results, sessions) is destroyed by an
# atexit hook, before the interpreter's module teardown and before the HIP runtime's own exit
# handlers: no fbn_* destroy ever runs from a finalizer racing those (or after `lib` is gone).
# Destroy order: results and sessions, then plans and contexts (they drain their device work),
# then host-only handles.
_LIVE = weakref.WeakSet()
_CLOSE_ORDER = {"PCResult": 0, "PCDistSession": 1, "JunctionTree": 2, "IndependenceTest": 3, "Dataset": 4,
                "Network": 5}


def _register(obj):
    _LIVE.add(obj)


def close_all():
    """Destroy every live handle now (also run at interpreter exit)."""
    objs = sorted(list(_LIVE), key=lambda o: _CLOSE_ORDER.get(type(o).__name__, 9))
    for o in objs:
        try:
            o.close()
        except Exception:  # noqa: BLE001 (exit path: keep closing the rest)
            pass


atexit.register(close_all)


class _Handle:
    """A libfastbn handle: `_h`, destroyed once by close() (explicitly, by __del__, or at exit)."""
    _destroy = None

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            getattr(lib, self._destroy)(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (finalizer)
            pass


def _p(a):
    return None if a is None else a.ctypes.data


def device_count():
    n = C.c_int(0)
    lib.fbn_device_count(C.byref(n))
    return n.value


class _PlanInfo(C.Structure):
    _fields_ = [("num_nodes", C.c_int32), ("num_cliques", C.c_int32), ("num_separators", C.c_int32),
                ("num_levels", C.c_int32), ("root", C.c_int32), ("sum_dom", C.c_int32),
                ("clique_entries", C.c_int64), ("separator_entries", C.c_int64),
                ("algorithmic_bytes_per_case", C.c_int64), ("num_ops", C.c_int32),
                ("max_vars_per_table", C.c_int32), ("specialized_eligible", C.c_int32),
                ("variant", C.c_int32), ("streamed_eligible", C.c_int32), ("streamed_waves", C.c_int32),
                ("streamed_split_efficiency", C.c_double), ("tiled_eligible", C.c_int32),
                ("tiled_passes", C.c_int32), ("tiled_entry_visits", C.c_int64), ("tiled_lds_bytes", C.c_int64),
                ("tiled_table_bytes", C.c_int64)]


class Network(_Handle):
    """Discrete BN loaded from XMLBIF (CustomNetwork::GetNetFromXMLBIFFile)."""

    _destroy = "fbn_network_destroy"

    def __init__(self, path=None, _handle=None):
        h = C.c_void_p() if _handle is None else _handle
        if _handle is None:
            lib.fbn_network_load_xmlbif(os.fsencode(path), C.byref(h))
        self._h = h
        _register(self)
        n = C.c_int()
        lib.fbn_network_num_nodes(h, C.byref(n))
        self.num_nodes = n.value
        self.dims = np.zeros(self.num_nodes, np.int32)
        lib.fbn_network_dims(h, _p(self.dims))

    @classmethod
    def from_counts(cls, dims, parents, counts, names=None):
        """A network built in memory (fbn_network_create; the reference's Network of DiscreteNodes,
        src/DiscreteNode.cpp:114-147): dims[v] states, parents[v] (the node's own order), counts[v]
        = int [dims[v]][parent configs], configurations over the parents in ascending index order,
        last fastest (map_cond_prob_table_statistics)."""
        n = len(dims)
        d = np.ascontiguousarray(dims, np.int32)
        off = np.zeros(n + 1, np.int32)
        for v in range(n):
            off[v + 1] = off[v] + len(parents[v])
        par = np.ascontiguousarray([q for ps in parents for q in ps] or [0], np.int32)
        cnt = np.ascontiguousarray(np.concatenate([np.asarray(c, np.int64).reshape(-1) for c in counts]), np.int64)
        nm = None
        if names is not None:
            enc = [os.fsencode(x) for x in names]
            nm = (C.c_char_p * n)(*enc)
        h = C.c_void_p()
        lib.fbn_network_create(n, _p(d), _p(off), _p(par), _p(cnt), C.cast(nm, C.c_void_p) if nm is not None else None,
                               C.byref(h))
        return cls(_handle=h)

    def node_counts(self, v):
        """(parents ascending, counts [dims[v]][parent configs]) of node v."""
        npar, ncnt = C.c_int(), C.c_int64()
        lib.fbn_network_node_counts(self._h, int(v), None, None, C.byref(npar), C.byref(ncnt))
        par = np.zeros(max(1, npar.value), np.int32)
        cnt = np.zeros(max(1, ncnt.value), np.int64)
        lib.fbn_network_node_counts(self._h, int(v), _p(par), _p(cnt), C.byref(npar), C.byref(ncnt))
        return par[:npar.value], cnt[:ncnt.value].reshape(int(self.dims[v]), -1)

    def name(self, i):
        buf = C.create_string_buffer(256)
        lib.fbn_network_name(self._h, i, buf, 256)
        return buf.value.decode()

    def forward_sample(self, n, seed):
        """n complete cases, uint8 [V][n] (fbn_synth_forward_sample; = synth.forward_sample)."""
        cols = np.empty((self.num_nodes, n), np.uint8)
        lib.fbn_synth_forward_sample(self._h, int(n), int(seed), _p(cols))
        return cols

    def evidence_cases(self, n, k, seed, query=0):
        """n evidence cases observing k variables each, int8 [n][V] (fbn_synth_evidence; =
        synth.evidence_cases)."""
        ev = np.empty((n, self.num_nodes), np.int8)
        lib.fbn_synth_evidence(self._h, int(n), int(k), int(seed), int(query), _p(ev))
        return ev



def write_csv(path, columns, network=None):
    """CSV of a column store (header + "s<code>" values), the reference's LoadCSVData input."""
    cols = np.ascontiguousarray(columns, np.uint8)
    lib.fbn_write_csv(os.fsencode(path), _p(cols), cols.shape[0], cols.shape[1], network._h if network else None)


def write_libsvm(path, evidence, labels=None):
    """LIBSVM test set of evidence rows (label + observed v:x), the reference's
    LoadLIBSVMDataKnownNetwork input."""
    ev = np.ascontiguousarray(evidence, np.int8)
    lab = None if labels is None else np.ascontiguousarray(labels, np.int32)
    lib.fbn_write_libsvm(os.fsencode(path), _p(ev), ev.shape[0], ev.shape[1], None if lab is None else _p(lab))


def kernel_options():
    """Compile options of the plan-specialized JT kernel (list of str)."""
    buf = C.create_string_buffer(1024)
    lib.fbn_jt_kernel_options(buf, 1024)
    return [x for x in buf.value.decode().split("\n") if x]


def load_libsvm(path, num_nodes):
    """Dataset::LoadLIBSVMDataKnownNetwork + Inference evidence extraction -> (evidence, labels)."""
    n = C.c_int64()
    lib.fbn_evidence_load_libsvm(os.fsencode(path), num_nodes, None, None, 0, C.byref(n))
    ev = np.zeros((n.value, num_nodes), np.int8)
    lab = np.zeros(n.value, np.int32)
    lib.fbn_evidence_load_libsvm(os.fsencode(path), num_nodes, _p(ev), _p(lab), n.value, C.byref(n))
    return ev, lab


class Dataset:
    """CSV training set with first-appearance value coding (Dataset::LoadCSVData)."""

    def __init__(self, path=None, columns=None, dims=None):
        if path is not None:
            h = C.c_void_p()
            lib.fbn_dataset_load_csv(os.fsencode(path), C.byref(h))
            nv, ns = C.c_int(), C.c_int64()
            lib.fbn_dataset_shape(h, C.byref(nv), C.byref(ns))
            self.dims = np.zeros(nv.value, np.int32)
            self.columns = np.zeros((nv.value, ns.value), np.uint8)
            lib.fbn_dataset_dims(h, _p(self.dims))
            lib.fbn_dataset_columns(h, _p(self.columns))
            self.names = []
            buf = C.create_string_buffer(256)
            for v in range(nv.value):
                lib.fbn_dataset_var_name(h, v, buf, 256)
                self.names.append(buf.value.decode())
            lib.fbn_dataset_destroy(h)
        else:
            self.columns = np.ascontiguousarray(columns, dtype=np.uint8)
            self.dims = np.ascontiguousarray(dims, dtype=np.int32)
            self.names = [str(i) for i in range(self.columns.shape[0])]

    @property
    def num_vars(self):
        return self.columns.shape[0]

    @property
    def num_instance(self):
        return self.columns.shape[1]


class JunctionTree(_Handle):
    """Batched JT inference on one device (JunctionTree ctor + PredictUseJTInfer over all cases)."""

    _destroy = "fbn_jt_plan_destroy"

    def __init__(self, network, device=0):
        self.network = network
        h = C.c_void_p()
        lib.fbn_jt_plan_create(network._h, device, C.byref(h))
        self._h = h
        _register(self)
        self.output_layout = 0
        info = _PlanInfo()
        lib.fbn_jt_plan_info_get(h, C.byref(info))
        self.info = {k: getattr(info, k) for k, _ in _PlanInfo._fields_}

    def tile_program(self):
        """The tiled kernel's program (variant 5): (passes [n][32] int32, tab int32, initv fp64,
        geometry dict) -- for host-side checks of its tables (tests/tile_emulator.py)."""
        g = np.zeros(8, np.int64)
        lib.fbn_jt_tile_program(self._h, None, None, None, _p(g))
        passes = np.zeros((int(g[0]), 33), np.int32)
        tab = np.zeros(max(int(g[1]), 1), np.int32)
        iv = np.zeros(max(int(g[2]), 1), np.float64)
        lib.fbn_jt_tile_program(self._h, _p(passes), _p(tab), _p(iv), _p(g))
        keys = ["n_passes", "n_tab", "n_init", "scr_row", "red_row", "store_rows", "cases_per_wave", "slots"]
        return passes, tab, iv, dict(zip(keys, (int(x) for x in g)))

    def dump_plan(self, plan_path, init_path):
        lib.fbn_jt_plan_dump(self._h, os.fsencode(plan_path), os.fsencode(init_path))

    def stream_schedule(self):
        """Streamed-kernel schedule: (order, sched) -- see fbn_jt_stream_schedule."""
        no, ns = C.c_int64(), C.c_int64()
        lib.fbn_jt_stream_schedule(self._h, None, 0, None, 0, C.byref(no), C.byref(ns))
        order = np.zeros(no.value, np.int32)
        sched = np.zeros(ns.value, np.int32)
        lib.fbn_jt_stream_schedule(self._h, _p(order), no.value, _p(sched), ns.value, None, None)
        return order, sched

    def set_waves_per_cu(self, w):
        lib.fbn_jt_set_waves_per_cu(self._h, w)

    def op_cycles(self, enable, read=True):
        """Diagnostic per-op-type cycles of the last run (LDS variant)."""
        buf = np.zeros(10, np.uint64)
        lib.fbn_jt_debug_op_cycles(self._h, int(enable), _p(buf) if read else None)
        names = ["INIT", "MUL", "SEPCOL", "STORE", "LOAD", "DMUL", "SEPDIS", "MARG", "EVZERO", "-"]
        return dict(zip(names, buf.tolist()))

    def kernel_source(self):
        """Source of the plan-specialized kernel (variant 3)."""
        n = C.c_int64()
        lib.fbn_jt_kernel_source(self._h, None, 0, C.byref(n))
        buf = C.create_string_buffer(n.value)
        lib.fbn_jt_kernel_source(self._h, buf, n.value, C.byref(n))
        return buf.value.decode()

    def kernel_cache_path(self):
        buf = C.create_string_buffer(4096)
        lib.fbn_jt_kernel_cache_path(self._h, buf, 4096)
        return buf.value.decode()

    def debug_force_fixup(self, enable):
        lib.fbn_jt_debug_force_fixup(self._h, int(enable))

    def debug_flagged_blocks(self):
        """64-case blocks the last run flagged for the exact fixup (variants 3-5)."""
        n = C.c_int64()
        lib.fbn_jt_debug_flagged_blocks(self._h, C.byref(n))
        return n.value

    def set_exact(self, exact):
        """Arithmetic order of the specialized / streamed kernels: True = the reference's
        (bit-identical), False = fast (normalizations that cancel left out; labels equal, marginals
        within 1e-12), None = auto (fast)."""
        lib.fbn_jt_set_exact(self._h, -1 if exact is None else int(bool(exact)))

    def build_kernel(self):
        """Compile the plan-specialized kernel into the on-disk cache (no GPU needed)."""
        lib.fbn_jt_kernel_build(self._h)
        return self.kernel_cache_path()

    def refresh_info(self):
        info = _PlanInfo()
        lib.fbn_jt_plan_info_get(self._h, C.byref(info))
        self.info = {k: getattr(info, k) for k, _ in _PlanInfo._fields_}
        return self.info

    def set_variant(self, v):
        """-1 auto, 0 = clique-in-LDS interpreter, 1 = global-workspace interpreter,
        2 = LDS interpreter with IEEE division, 3 = plan-specialized kernel,
        4 = streamed (virtual-table) kernel for large trees, 5 = per-case evidence-reduced
        kernel for large trees (fast arithmetic order)."""
        lib.fbn_jt_set_variant(self._h, v)

    def infer(self, evidence, marginals=True):
        """evidence [ncases][num_nodes] int8 (-1 unobserved) -> (labels, marginals or None)."""
        ev = np.ascontiguousarray(evidence, dtype=np.int8)
        n = ev.shape[0]
        labels = np.zeros(n, np.int32)
        marg = np.zeros((n, self.info["sum_dom"]), np.float64) if marginals else None
        lib.fbn_jt_run(self._h, _p(ev), n, _p(labels), _p(marg), None)
        return labels, marg

    def run_device(self, d_evidence_ptr, ncases, d_labels_ptr, d_marg_ptr, stream_ptr=None):
        """Device-resident run (asynchronous on the stream unless the evidence check is on)."""
        lib.fbn_jt_run_device(self._h, d_evidence_ptr, ncases, d_labels_ptr, d_marg_ptr, stream_ptr)

    def validate_device(self, d_evidence_ptr, ncases, stream_ptr=None):
        """Device-side evidence range check of a device buffer; raises FastBNError if a code is out
        of its node's domain."""
        lib.fbn_jt_evidence_validate(self._h, d_evidence_ptr, ncases, stream_ptr)

    def set_kernel_timing(self, enable):
        """fbn_jt_set_kernel_timing: enable = False records no timing events per run (last_kernel_ms
        then raises); for callers that time with their own events."""
        lib.fbn_jt_set_kernel_timing(self._h, int(bool(enable)))

    def set_evidence_check(self, enable):
        """run_device's per-call evidence check (default on); off = fully asynchronous runs of a
        buffer the caller validated (validate_device)."""
        lib.fbn_jt_set_evidence_check(self._h, int(bool(enable)))

    def set_output_layout(self, layout):
        """fbn_jt_set_output_layout: run_device's marginals 0 = case-major [ncases][sum_dom]
        (default), 1 = variable-major [sum_dom][ncases] (each store writes 64 consecutive cases).
        infer() always returns case-major."""
        lib.fbn_jt_set_output_layout(self._h, int(layout))
        self.output_layout = int(layout)

    def score_terms_device(self, d_marg_ptr, d_golden_ptr, ncases, d_terms_ptr, stream_ptr=None):
        """fbn_jt_score_terms_device: per-case (MSE, HD) terms [ncases][2] fp64 on the device from
        device marginals (the plan's output layout) and a case-major device golden table."""
        lib.fbn_jt_score_terms_device(self._h, d_marg_ptr, d_golden_ptr, ncases, d_terms_ptr, stream_ptr)

    def last_kernel_ms(self):
        ms = C.c_float()
        lib.fbn_jt_last_kernel_ms(self._h, C.byref(ms))
        return ms.value

    def score(self, marginals, golden):
        mse, hd = C.c_double(), C.c_double()
        m = np.ascontiguousarray(marginals, np.float64)
        g = np.ascontiguousarray(golden, np.float64)
        lib.fbn_jt_score(self._h, _p(m), _p(g), m.shape[0], C.byref(mse), C.byref(hd))
        return mse.value, hd.value

    def EvaluateAccuracy(self, evidence, ground_truths, golden=None):
        """Accuracy of the query-variable arg-max (+ average MSE/HD vs golden if given)."""
        labels, marg = self.infer(evidence)
        acc = float(np.mean(labels == np.asarray(ground_truths)))
        if golden is None:
            return acc
        mse, hd = self.score(marg, golden)
        return acc, mse / len(labels), hd / len(labels)



class IndependenceTest(_Handle):
    """G^2 tests on the device (IndependenceTest::IndependenceResult, batched)."""

    _destroy = "fbn_ci_ctx_destroy"

    def __init__(self, dataset, alpha=0.05, device=0):
        self.alpha = alpha
        self.dims = np.ascontiguousarray(dataset.dims, np.int32)
        h = C.c_void_p()
        lib.fbn_ci_dataset_upload(_p(dataset.columns), dataset.num_vars, dataset.num_instance,
                                  _p(dataset.dims), device, C.byref(h))
        self._h = h
        _register(self)

    @classmethod
    def from_device(cls, d_cols_ptr, nvars, nsamples, dims, alpha=0.05, device=0):
        """Column store already in `device` memory (uint8 [nvars][nsamples], e.g. a tensor filled by
        an RCCL broadcast): fbn_ci_dataset_from_device."""
        self = cls.__new__(cls)
        self.alpha = alpha
        dims = np.ascontiguousarray(dims, np.int32)
        self.dims = dims
        h = C.c_void_p()
        lib.fbn_ci_dataset_from_device(C.c_void_p(d_cols_ptr), int(nvars), int(nsamples), _p(dims), device,
                                       C.byref(h))
        self._h = h
        _register(self)
        return self

    def set_kernel_timing(self, enable):
        """HIP-event kernel timing of every CI launch (default on; off saves the events' cost)."""
        lib.fbn_ci_set_kernel_timing(self._h, int(bool(enable)))

    def level(self, d, edges, e_begin, e_end, group_size=1):
        """One skeleton level for edges[e_begin:e_end] of the current skeleton (fbn_pc_level) ->
        (removed[bool], sepsets[list of tuples or None], counted, launched)."""
        ev = np.ascontiguousarray(np.asarray(edges, np.int32).reshape(-1, 2))
        n = e_end - e_begin
        rm = np.zeros(max(n, 1), np.uint8)
        sp = np.zeros((max(n, 1), max(d, 1)), np.int32)
        cnt, lau = C.c_int64(), C.c_int64()
        lib.fbn_pc_level(self._h, self.alpha, d, group_size, _p(ev), ev.shape[0], e_begin, e_end, _p(rm), _p(sp),
                         C.byref(cnt), C.byref(lau))
        rm = rm[:n].astype(bool)
        seps = [tuple(int(v) for v in sp[i, :d]) if rm[i] else None for i in range(n)]
        return rm, seps, cnt.value, lau.value

    def run(self, items, d):
        items = np.ascontiguousarray(items, dtype=np.int32).reshape(-1, 2 + d)
        n = items.shape[0]
        g2 = np.zeros(n)
        df = np.zeros(n, np.int32)
        p = np.zeros(n)
        ind = np.zeros(n, np.uint8)
        lib.fbn_ci_run(self._h, _p(items), n, d, self.alpha, _p(g2), _p(df), _p(p), _p(ind), None)
        return g2, df, p, ind.astype(bool)

    def IndependenceResult(self, x, y, z=()):
        g2, df, p, ind = self.run(np.array([[x, y, *z]], np.int32), len(z))
        return {"g2": g2[0], "df": int(df[0]), "p_value": p[0], "is_independent": bool(ind[0])}

    def production_counts(self, items, d, cap=None):
        """Counts of the tests `items` [n][2+d] through the kernels a PC run uses at level d
        (fbn_ci_debug_counts: level-0 Gram + pair tables, derived level-1 counting, histogram
        kernel) -> int32 [n][cap] (Counts3D order; cells beyond a test's table are 0)."""
        items = np.ascontiguousarray(items, np.int32).reshape(-1, 2 + d)
        if cap is None:
            dims = np.asarray(self.dims)
            cap = int(np.max(np.prod(dims[items], axis=1))) if len(items) else 1
        out = np.zeros((len(items), cap), np.int32)
        lib.fbn_ci_debug_counts(self._h, _p(items), len(items), d, _p(out), cap)
        return out

    def counts(self, x, y, z=()):
        zz = np.array(z, np.int32)
        cells = C.c_int64()
        lib.fbn_ci_counts(self._h, x, y, _p(zz) if len(z) else None, len(z), None, 0, C.byref(cells))
        out = np.zeros(cells.value, np.int32)
        lib.fbn_ci_counts(self._h, x, y, _p(zz) if len(z) else None, len(z), _p(out), cells.value,
                          C.byref(cells))
        return out

    def decision_margin(self, reset=False):
        """(min |p - alpha|, #tests with |p - alpha| < 1e-9) over the tests run since the last reset."""
        m, near = C.c_double(), C.c_int64()
        lib.fbn_ci_decision_margin(self._h, C.byref(m), C.byref(near), int(bool(reset)))
        return m.value, near.value

    def last_kernel_ms(self):
        ms = C.c_float()
        lib.fbn_ci_last_kernel_ms(self._h, C.byref(ms))
        return ms.value



class PCResult(_Handle):
    """A PC-stable result handle: skeleton, sepsets, orientation, SHD (fbn_pc_*)."""

    _destroy = "fbn_pc_result_destroy"

    def __init__(self, handle):
        self._h = handle
        _register(self)
        self._edges = self._sepset = self._oriented = None
        m, near = C.c_double(), C.c_int64()
        lib.fbn_pc_decision_margin(handle, C.byref(m), C.byref(near))
        # p-values are parity-unpinned; decisions this close to alpha are flagged
        self.min_margin, self.near_alpha = m.value, near.value
        nl = C.c_int()
        lib.fbn_pc_num_levels(handle, C.byref(nl))
        self.tests_per_level = np.zeros(nl.value, np.int64)
        self.launched_per_level = np.zeros(nl.value, np.int64)
        if nl.value:
            lib.fbn_pc_level_tests(handle, _p(self.tests_per_level))
            lib.fbn_pc_level_launched(handle, _p(self.launched_per_level))
        self.num_ci_test = int(self.tests_per_level.sum())
        tot, ker = C.c_double(), C.c_double()
        lib.fbn_pc_timing(handle, C.byref(tot), C.byref(ker))
        self.total_s, self.kernel_s = tot.value, ker.value
        path = C.c_int()
        lib.fbn_pc_path(handle, C.byref(path))
        # 0 host-driven levels, 1 device-resident search, 2 device-resident search fell back to the host
        self.path = path.value
        nb = C.c_int64()
        lib.fbn_pc_device_bytes(handle, C.byref(nb))
        self.device_bytes = nb.value

    @classmethod
    def with_levels(cls, handle):
        return cls(handle)

    # skeleton / sepsets / orientation are converted to Python objects on first access (a
    # 1000-variable run has ~500k sepsets: the conversion costs far more than the search)
    @property
    def edges(self):
        if self._edges is None:
            ne = C.c_int()
            lib.fbn_pc_num_edges(self._h, C.byref(ne))
            e = np.zeros((max(ne.value, 1), 2), np.int32)
            if ne.value:
                lib.fbn_pc_edges(self._h, _p(e))
            self._edges = [tuple(map(int, x)) for x in e[:ne.value]]
        return self._edges

    @property
    def sepset(self):
        if self._sepset is None:
            ln = C.c_int64()
            lib.fbn_pc_sepsets(self._h, None, 0, C.byref(ln))
            buf = np.zeros(max(ln.value, 1), np.int32)
            lib.fbn_pc_sepsets(self._h, _p(buf), ln.value, C.byref(ln))
            sep, k, b = {}, 0, buf.tolist()
            while k < ln.value:
                x, y, m = b[k], b[k + 1], b[k + 2]
                sep[(x, y)] = tuple(b[k + 3:k + 3 + m])
                k += 3 + m
            self._sepset = sep
        return self._sepset

    @property
    def oriented(self):
        """(from, to, 1) arcs and (min, max, 0) undirected edges, in vec_edges order."""
        if self._oriented is None:
            no = C.c_int()
            lib.fbn_pc_num_oriented_edges(self._h, C.byref(no))
            t = np.zeros((max(no.value, 1), 3), np.int32)
            if no.value:
                lib.fbn_pc_oriented_edges(self._h, _p(t))
            self._oriented = [tuple(map(int, x)) for x in t[:no.value]]
        return self._oriented

    def GetSHD(self, bif_path):
        """BNSLComparison(ref_net, network).GetSHD() with ref_net loaded from a BIF file."""
        shd = C.c_int()
        lib.fbn_pc_shd_bif(self._h, os.fsencode(bif_path), C.byref(shd))
        return shd.value



def shd_bif(bif_path, nvars, oriented):
    """SHD of a learned graph [(from, to, 1) | (a, b, 0)] vs the CPDAG of a BIF DAG."""
    t = np.ascontiguousarray(np.asarray(oriented if oriented else [(0, 0, 0)], np.int32).reshape(-1, 3))
    shd = C.c_int()
    lib.fbn_shd_bif(os.fsencode(bif_path), int(nvars), _p(t), len(oriented), C.byref(shd))
    return shd.value


def orient_skeleton(nvars, edges, sepset):
    """Host-only orientation of a given skeleton (PCStable steps 2-3) -> PCResult."""
    pairs = np.ascontiguousarray(np.asarray(edges, np.int32).reshape(-1, 2))
    rec = []
    for (x, y), z in sorted(sepset.items()):
        rec += [x, y, len(z)] + list(z)
    rec = np.ascontiguousarray(np.asarray(rec if rec else [0], np.int32))
    r = C.c_void_p()
    lib.fbn_pc_orient_skeleton(int(nvars), _p(pairs), int(pairs.shape[0]), _p(rec), len(rec) if sepset else 0,
                               C.byref(r))
    return PCResult(r)


class PCStable:
    """PC-stable (PCStable(net, alpha, depth).StructLearnCompData): device skeleton + host orientation."""

    def __init__(self, alpha=0.05, depth=1000, device=0):
        self.alpha, self.depth, self.device = alpha, depth, device
        self.result = None

    def StructLearnCompData(self, dataset, group_size=1, num_threads=1, print_struct=False, verbose=False):
        """`dataset`: a Dataset (uploaded for this call) or an IndependenceTest whose column store is
        already resident on the device (reused across calls)."""
        ci = dataset if isinstance(dataset, IndependenceTest) else IndependenceTest(dataset, self.alpha, self.device)
        r = C.c_void_p()
        lib.fbn_pc_stable(ci._h, self.alpha, self.depth, group_size, C.byref(r))
        self.result = res = PCResult(r)
        self.tests_per_level, self.launched_per_level = res.tests_per_level, res.launched_per_level
        self.total_s, self.kernel_s, self.device_bytes = res.total_s, res.kernel_s, res.device_bytes
        self.num_ci_test = res.num_ci_test
        self.min_margin, self.near_alpha = self.result.min_margin, self.result.near_alpha
        return self

    edges = property(lambda self: self.result.edges)
    sepset = property(lambda self: self.result.sepset)
    oriented = property(lambda self: self.result.oriented)
    path = property(lambda self: self.result.path)  # 0 host levels, 1 device-resident, 2 fell back, 3 host levels after the device level 0 -> 1 hand-off

    def GetSHD(self, bif_path):
        return self.result.GetSHD(bif_path)
