"""ctypes wrapper of the CPU oracle (oracle/_build/liblvg_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package. Parity unpinned —
see lvg_oracle.c's header.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from radiative_transfer_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liblvg_oracle.so")
# reference-arithmetic builds: -DORACLE_REF_ARITH (glibc exp/log10/pow, LU without fma)
# and one build per choice (-DORACLE_REF_EXP, _LU, _POW); ref= selects one by name
REF_MASK = {False: 0, None: 0, True: 7, "all": 7, "exp": 1, "lu": 2, "pow": 4}
REF_LIB = {0: LIB_PATH, 7: os.path.join(HERE, "_build", "liblvg_oracle_ref.so"),
           1: os.path.join(HERE, "_build", "liblvg_oracle_ref_exp.so"),
           2: os.path.join(HERE, "_build", "liblvg_oracle_ref_lu.so"),
           4: os.path.join(HERE, "_build", "liblvg_oracle_ref_pow.so")}
REF_LIB_PATH = REF_LIB[7]
_libs = {}
# the CPU timing leg (bench.py cpu_baseline): reference arithmetic, -O3 -march=native -fopenmp,
# contraction allowed; built per host CPU model, since -march=native code must not move
NATIVE_FLAGS = "-O3 -march=native -fopenmp -DORACLE_REF_ARITH (fp contraction allowed)"


def _cpu_tag() -> str:
    import hashlib
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith(("model name", "flags")):
                    model += line
    except OSError:
        pass
    return hashlib.sha1(model.encode()).hexdigest()[:12]


def native_lib_path() -> str:
    return os.path.join(HERE, "_build", "native", _cpu_tag(), "liblvg_oracle_native.so")


def build_native() -> str:
    p = native_lib_path()
    subprocess.check_call(["make", "-s", "-C", HERE, "native", f"NATIVE_OUT={os.path.dirname(p)}"])
    return p


def _stale() -> bool:
    if not all(os.path.exists(p) for p in REF_LIB.values()):
        return True
    t = min(os.path.getmtime(p) for p in REF_LIB.values())
    deps = [os.path.join(HERE, f) for f in ("lvg_oracle.c", "lvg_oracle.h", "Makefile")]
    deps += [os.path.join(HERE, "..", "include", f) for f in ("lvg_amd.h", "lvg_math.h")]
    return any(os.path.getmtime(x) > t for x in deps)


def build(force: bool = False) -> str:
    if force or _stale():
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib(ref=False):
    """The bit-exact oracle, or with ref=True its reference-arithmetic build; ref="exp",
    "lu" or "pow" undoes that one choice only; ref="native" is the CPU timing leg's build
    (reference arithmetic, -march=native, contraction allowed: not a checker)."""
    key = ref if ref == "native" else REF_MASK[ref]
    mask = 7 if ref == "native" else key
    if key not in _libs:
        if ref == "native":
            L = C.CDLL(build_native())
        else:
            build()
            L = C.CDLL(REF_LIB[mask])
        d, i, vp = C.c_double, C.c_int, C.c_void_p
        dp = C.POINTER(C.c_double)
        L.oracle_solve_layers.argtypes = [vp, vp, dp, vp, vp, i]
        L.oracle_solve_chains.argtypes = [vp, vp, i, C.POINTER(C.c_int), dp, vp, vp, i]
        L.oracle_calc_new_pop.argtypes = [vp, vp, i, dp, i, dp, dp, dp, dp]
        L.oracle_boundary_layer_populations.argtypes = [vp, vp, dp]
        L.oracle_coll_rates.argtypes = [vp, vp, i, dp, dp, dp, dp]
        L.oracle_line_groups.argtypes = [vp, C.POINTER(C.c_int), i]
        L.oracle_nb_overlap_lines.argtypes = [vp, d, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_esc_func.argtypes = [vp, d, d]
        L.oracle_esc_func.restype = d
        L.oracle_overlap_esc_func.argtypes = [vp, d, d, d, d]
        L.oracle_overlap_esc_func.restype = d
        L.oracle_dust_absorption.argtypes = [vp, d, dp]
        L.oracle_dust_absorption.restype = d
        L.oracle_lu_solve.argtypes = [dp, dp, i]
        L.oracle_find_transitions.argtypes = [vp, vp, vp, dp, vp, i, C.POINTER(C.c_int), vp, dp, dp, dp]
        ipp = C.POINTER(C.c_int)
        L.oracle_lim_luminosity.argtypes = [vp, vp, vp, dp, i, ipp, ipp, i, dp, dp, dp, dp, dp, dp]
        L.oracle_exp.argtypes = [d]
        L.oracle_exp.restype = d
        L.oracle_log10.argtypes = [d]
        L.oracle_log10.restype = d
        L.oracle_ref_arith.restype = i
        assert L.oracle_ref_arith() == mask
        _libs[key] = L
    return _libs[key]


def _nz(a):
    return abi.dptr(a) if a is not None else None


def solve_layers(prob: abi.Problem, layers: abi.Layers, opts=None, pops=None, nthreads: int = 0, ref=False):
    cp, cl = prob.to_c(), layers.to_c()
    N = prob.mol.nb_lev
    o = opts if opts is not None else abi.default_opts()
    out = np.zeros((layers.nb_lay, N)) if pops is None else np.array(pops, dtype=np.float64, copy=True)
    st = np.zeros(layers.nb_lay, dtype=abi.STATUS_DTYPE)
    rc = lib(ref).oracle_solve_layers(cp.ptr, cl.ptr, abi.dptr(out), C.byref(o),
                                   st.ctypes.data_as(C.c_void_p), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_solve_layers failed: {rc}")
    return out, st


def solve_chains(prob: abi.Problem, layers: abi.Layers, chain_off, opts=None, nthreads: int = 0, ref=False):
    """oracle_solve_chains: independent warm chains [chain_off[c], chain_off[c+1])."""
    cp, cl = prob.to_c(), layers.to_c()
    o = opts if opts is not None else abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN)
    off = np.ascontiguousarray(chain_off, dtype=np.int32)
    out = np.zeros((layers.nb_lay, prob.mol.nb_lev))
    st = np.zeros(layers.nb_lay, dtype=abi.STATUS_DTYPE)
    rc = lib(ref).oracle_solve_chains(cp.ptr, cl.ptr, len(off) - 1, off.ctypes.data_as(C.POINTER(C.c_int)),
                                      abi.dptr(out), C.byref(o), st.ctypes.data_as(C.c_void_p), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_solve_chains failed: {rc}")
    return out, st


def calc_new_pop(prob, layers, layer, pop_in, overlap=0, ref=False):
    cp, cl = prob.to_c(), layers.to_c()
    N = prob.mol.nb_lev
    pin = np.ascontiguousarray(pop_in, dtype=np.float64)
    M = np.zeros((N, N)); df = np.zeros(N); pout = np.zeros(N); e = C.c_double()
    rc = lib(ref).oracle_calc_new_pop(cp.ptr, cl.ptr, layer, abi.dptr(pin), overlap, abi.dptr(M),
                                   abi.dptr(df), abi.dptr(pout), C.byref(e))
    assert rc == 0
    return M, df, pout, e.value


def boundary_layer_populations(prob, layers, ref=False):
    cp, cl = prob.to_c(), layers.to_c()
    out = np.zeros((layers.nb_lay, prob.mol.nb_lev))
    lib(ref).oracle_boundary_layer_populations(cp.ptr, cl.ptr, abi.dptr(out))
    return out


def coll_rates(prob, layers, layer):
    cp, cl = prob.to_c(), layers.to_c()
    N = prob.mol.nb_lev
    a = [np.zeros((N, N)) for _ in range(4)]
    lib().oracle_coll_rates(cp.ptr, cl.ptr, layer, *[abi.dptr(x) for x in a])
    return a


def line_groups(prob):
    cp = prob.to_c()
    N = prob.mol.nb_lev
    g = np.zeros((N * N, 5), dtype=np.int32)
    n = lib().oracle_line_groups(cp.ptr, g.ctypes.data_as(C.POINTER(C.c_int)), N * N)
    assert n >= 0
    return g[:n].copy()


def esc_func(prob, gamma, delta):
    cp = prob.to_c()
    return lib().oracle_esc_func(C.byref(cp.esc), gamma, delta)


def overlap_esc_func(prob, which, gamma, delta, gratio, dx):
    cp = prob.to_c()
    return lib().oracle_overlap_esc_func(C.byref(cp.ov[which]), gamma, delta, gratio, dx)


def lu_solve(a, b):
    a = np.array(a, dtype=np.float64, copy=True)
    b = np.array(b, dtype=np.float64, copy=True)
    lib().oracle_lu_solve(abi.dptr(a), abi.dptr(b), b.size)
    return b


def find_transitions(prob, layers, geo, pops, opts=None, max_out: int = 256):
    """oracle_find_transitions: same outputs as LvgSolver.find_transitions."""
    cp, cl = prob.to_c(), layers.to_c()
    cg = geo.to_c()
    o = opts if opts is not None else abi.find_opts()
    p = np.ascontiguousarray(pops, dtype=np.float64)
    nl = layers.nb_lay
    while True:
        out = np.zeros(max_out, dtype=abi.TRANSITION_DTYPE)
        inv = np.zeros((max_out, nl)); gain = np.zeros((max_out, nl)); exc = np.zeros((max_out, nl))
        n = C.c_int()
        rc = lib().oracle_find_transitions(cp.ptr, cl.ptr, C.byref(cg), abi.dptr(p), C.byref(o), max_out, C.byref(n),
                                           out.ctypes.data_as(C.c_void_p), abi.dptr(inv), abi.dptr(gain), abi.dptr(exc))
        assert rc == 0
        if n.value <= max_out:
            k = n.value
            return out[:k].copy(), inv[:k].copy(), gain[:k].copy(), exc[:k].copy()
        max_out = n.value


def lim_luminosity(prob, layers, geo, pops, up, low, layer_pops: int = 0):
    """oracle_lim_luminosity: same outputs as LvgSolver.lim_luminosity."""
    from radiative_transfer_amd.native import _lim_lum_call
    cp = prob.to_c()

    def check(rc):
        assert rc == 0
    return _lim_lum_call(lib().oracle_lim_luminosity, check, cp.ptr, layers, geo, pops, up, low, layer_pops)

