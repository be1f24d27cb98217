"""TEST INFRASTRUCTURE: ctypes wrapper of oracle/liboracle.so (CPU restatement of the reference).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / reported baseline -- never as the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_vp, _i64, _dbl = C.c_void_p, C.c_int64, C.c_double


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def _load():
    if not os.path.exists(LIB):
        build()
    L = C.CDLL(LIB)
    sig = {
        "or_jt_load": ([C.c_char_p], _vp), "or_jt_destroy": ([_vp], None), "or_jt_nvars": ([_vp], C.c_int),
        "or_jt_dims": ([_vp, _vp], C.c_int), "or_jt_dump_plan": ([_vp, C.c_char_p, C.c_char_p], C.c_int),
        "or_jt_infer": ([_vp, _vp, _i64, _vp, _vp], C.c_int), "or_round7": ([_dbl], _dbl),
        "or_libsvm_load": ([C.c_char_p, C.c_int, _vp, _vp, _i64], _i64),
        "or_csv_load": ([C.c_char_p], _vp), "or_ds_from_columns": ([_vp, C.c_int, _i64, _vp], _vp),
        "or_ds_destroy": ([_vp], None), "or_ds_shape": ([_vp, _vp, _vp], C.c_int),
        "or_ds_dims": ([_vp, _vp], C.c_int), "or_ds_columns": ([_vp, _vp], C.c_int),
        "or_chisq_pvalue": ([_dbl, C.c_int], _dbl),
        "or_ci_test": ([_vp, C.c_int, C.c_int, _vp, C.c_int, _dbl, _vp, _vp, _vp, _vp, _vp, _i64], C.c_int),
        "or_pc_run": ([_vp, _dbl, C.c_int, C.c_int, C.c_int], _vp), "or_pc_destroy": ([_vp], None),
        "or_pc_num_ci": ([_vp], _i64), "or_pc_levels": ([_vp, _vp, C.c_int], C.c_int),
        "or_pc_edges": ([_vp, _vp, C.c_int], C.c_int), "or_pc_sepsets": ([_vp, _vp, _i64], _i64),
        "or_pc_log_size": ([_vp], _i64),
        "or_pc_log_entry": ([_vp, _i64, _vp, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    }
    for k, (a, r) in sig.items():
        f = getattr(L, k)
        f.argtypes, f.restype = a, r
    return L


_L = None


def L():
    global _L
    if _L is None:
        _L = _load()
    return _L


class OracleJT:
    def __init__(self, xml_path):
        self.h = L().or_jt_load(os.fsencode(xml_path))
        self.n = L().or_jt_nvars(self.h)
        d = (C.c_int * self.n)()
        L().or_jt_dims(self.h, d)
        self.dims = np.array(list(d), np.int32)
        self.sum_dom = int(self.dims.sum())

    def dump_plan(self, plan, init):
        L().or_jt_dump_plan(self.h, os.fsencode(plan), os.fsencode(init))

    def infer(self, evidence):
        ev = np.ascontiguousarray(evidence, np.int8)
        n = ev.shape[0]
        marg = np.zeros((n, self.sum_dom))
        lab = np.zeros(n, np.int32)
        L().or_jt_infer(self.h, ev.ctypes.data, n, marg.ctypes.data, lab.ctypes.data)
        return lab, marg

    def __del__(self):
        if getattr(self, "h", None):
            L().or_jt_destroy(self.h)
            self.h = None


def load_libsvm(path, n):
    cnt = L().or_libsvm_load(os.fsencode(path), n, None, None, 0)
    ev = np.zeros((cnt, n), np.int8)
    lab = np.zeros(cnt, np.int32)
    L().or_libsvm_load(os.fsencode(path), n, ev.ctypes.data, lab.ctypes.data, cnt)
    return ev, lab


class OracleDataset:
    def __init__(self, csv=None, columns=None, dims=None):
        if csv is not None:
            self.h = L().or_csv_load(os.fsencode(csv))
        else:
            cols = np.ascontiguousarray(columns, np.uint8)
            dd = np.ascontiguousarray(dims, np.int32)
            self.h = L().or_ds_from_columns(cols.ctypes.data, cols.shape[0], cols.shape[1], dd.ctypes.data)
        nv, ns = C.c_int(), C.c_int64()
        L().or_ds_shape(self.h, C.byref(nv), C.byref(ns))
        self.dims = np.zeros(nv.value, np.int32)
        L().or_ds_dims(self.h, self.dims.ctypes.data)
        self.columns = np.zeros((nv.value, ns.value), np.uint8)
        L().or_ds_columns(self.h, self.columns.ctypes.data)

    def ci_test(self, x, y, z=(), alpha=0.05, counts=False):
        zz = np.array(z, np.int32)
        g2, df, p, ind = C.c_double(), C.c_int32(), C.c_double(), C.c_int32()
        buf = None
        if counts:
            cells = int(self.dims[x] * self.dims[y] * np.prod([self.dims[v] for v in z] or [1]))
            buf = np.zeros(cells, np.int32)
        L().or_ci_test(self.h, x, y, zz.ctypes.data if len(z) else None, len(z), alpha, C.byref(g2),
                       C.byref(df), C.byref(p), C.byref(ind), None if buf is None else buf.ctypes.data,
                       0 if buf is None else buf.size)
        r = {"g2": g2.value, "df": df.value, "p_value": p.value, "is_independent": bool(ind.value)}
        if counts:
            r["counts"] = buf
        return r

    def pc_stable(self, alpha=0.05, depth=1000, group_size=1, keep_log=False):
        r = L().or_pc_run(self.h, alpha, depth, group_size, int(keep_log))
        try:
            lv = np.zeros(64, np.int64)
            nl = L().or_pc_levels(r, lv.ctypes.data, 64)
            e = np.zeros((self.dims.size * self.dims.size, 2), np.int32)
            ne = L().or_pc_edges(r, e.ctypes.data, e.shape[0])
            ln = L().or_pc_sepsets(r, None, 0)
            buf = np.zeros(max(ln, 1), np.int32)
            L().or_pc_sepsets(r, buf.ctypes.data, ln)
            sep, k = {}, 0
            while k < ln:
                x, y, m = map(int, buf[k:k + 3])
                sep[(x, y)] = tuple(int(v) for v in buf[k + 3:k + 3 + m])
                k += 3 + m
            log = []
            if keep_log:
                ints = np.zeros(4 + 16, np.int32)
                g2, df, p, ind = C.c_double(), C.c_int32(), C.c_double(), C.c_int32()
                for i in range(L().or_pc_log_size(r)):
                    L().or_pc_log_entry(r, i, ints.ctypes.data, 16, C.byref(g2), C.byref(df), C.byref(p),
                                        C.byref(ind))
                    d = int(ints[3])
                    log.append((int(ints[0]), int(ints[1]), int(ints[2]), tuple(int(v) for v in ints[4:4 + d]),
                                g2.value, df.value, p.value, bool(ind.value)))
            return {"tests_per_level": lv[:nl].tolist(), "edges": [tuple(map(int, x)) for x in e[:ne]],
                    "sepset": sep, "num_ci_test": int(L().or_pc_num_ci(r)), "log": log}
        finally:
            L().or_pc_destroy(r)

    def __del__(self):
        if getattr(self, "h", None):
            L().or_ds_destroy(self.h)
            self.h = None


def chisq_pvalue(g2, df):
    return L().or_chisq_pvalue(g2, df)


def round7(x):
    return L().or_round7(x)
