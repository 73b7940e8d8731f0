"""ctypes binding of liblvg_amd.so (the C ABI of include/lvg_amd.h).

There is no CPU fallback: if the HIP library is missing or cannot load, every
entry point raises. This is the same binding a maintainer would add on the
reference side.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LVG_LIB_PATH") or os.path.join(_PKG, "_lib", "liblvg_amd.so")

# every symbol include/lvg_amd.h declares
EXPORTS = ("lvg_abi_version", "lvg_solve_opts_default", "lvg_create", "lvg_destroy", "lvg_last_error",
           "lvg_nb_lev", "lvg_solve_layers", "lvg_layer_soa_rows", "lvg_solve_layers_device",
           "lvg_debug_calc_new_pop", "lvg_boundary_layer_populations", "lvg_find_opts_default",
           "lvg_find_transitions", "lvg_lim_luminosity", "lvg_last_kernel_time", "lvg_solve_chains",
           "lvg_solve_chains_device", "lvg_last_coll_time", "lvg_set_tuning", "lvg_last_kernel_kind",
           "lvg_create_multi", "lvg_create_devices", "lvg_nb_devices", "lvg_shard_range", "lvg_chain_shard")

_lib = None


class LvgError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load the library (no device work). Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise LvgError(f"HIP library not built: {path} (run radiative_transfer_amd.build)")
    L = C.CDLL(path)
    vp, i, dp = C.c_void_p, C.c_int, C.POINTER(C.c_double)
    L.lvg_abi_version.restype = i
    L.lvg_solve_opts_default.argtypes = [vp]
    L.lvg_create.argtypes = [vp, i, C.POINTER(vp)]
    L.lvg_destroy.argtypes = [vp]
    L.lvg_last_error.argtypes = [vp]
    L.lvg_last_error.restype = C.c_char_p
    L.lvg_nb_lev.argtypes = [vp]
    L.lvg_solve_layers.argtypes = [vp, vp, dp, vp, vp]
    L.lvg_layer_soa_rows.argtypes = [vp]
    L.lvg_solve_layers_device.argtypes = [vp, i, vp, vp, vp, vp, vp]
    L.lvg_solve_chains.argtypes = [vp, vp, i, C.POINTER(C.c_int), dp, vp, vp]
    L.lvg_solve_chains_device.argtypes = [vp, i, vp, i, C.POINTER(C.c_int), vp, vp, vp, vp]
    L.lvg_debug_calc_new_pop.argtypes = [vp, vp, i, dp, i, dp, dp, dp, dp]
    L.lvg_boundary_layer_populations.argtypes = [vp, vp, dp]
    L.lvg_last_kernel_time.argtypes = [vp, dp, C.POINTER(C.c_int)]
    L.lvg_last_coll_time.argtypes = [vp, dp]
    L.lvg_set_tuning.argtypes = [vp, C.c_char_p]
    L.lvg_last_kernel_kind.argtypes = [vp, C.POINTER(C.c_int)]
    L.lvg_find_opts_default.argtypes = [vp]
    L.lvg_create_multi.argtypes = [vp, C.c_uint, C.POINTER(vp)]
    L.lvg_create_devices.argtypes = [vp, i, C.POINTER(C.c_int), C.POINTER(vp)]
    L.lvg_nb_devices.argtypes = [vp]
    L.lvg_shard_range.argtypes = [i, i, i, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.lvg_chain_shard.argtypes = [i, C.POINTER(C.c_int), i, i, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    ip = C.POINTER(C.c_int)
    L.lvg_lim_luminosity.argtypes = [vp, vp, vp, dp, i, ip, ip, i, dp, dp, dp, dp, dp, dp]
    L.lvg_find_transitions.argtypes = [vp, vp, vp, dp, vp, i, C.POINTER(C.c_int), vp, dp, dp, dp]
    _lib = L
    return L


class LvgSolver:
    """One handle: the device-resident tables of one molecule (lvg_create).

    Mirrors the reference object graph built before calc_molecular_populations
    (energy_diagram, einstein_coeff, collisional_transitions, iteration_scheme_lvg).
    """

    def __init__(self, problem: abi.Problem, device: int = 0, devices=None, device_mask: int = 0):
        """One device (lvg_create), or several in this process: `devices` (lvg_create_devices,
        repeats allowed) or `device_mask` (lvg_create_multi)."""
        self.lib = load()
        self.problem = problem
        self.N = problem.mol.nb_lev
        self._cp = problem.to_c()
        h = C.c_void_p()
        if devices is not None:
            d = np.ascontiguousarray(devices, dtype=np.int32)
            rc = self.lib.lvg_create_devices(self._cp.ptr, len(d), d.ctypes.data_as(C.POINTER(C.c_int)), C.byref(h))
        elif device_mask:
            rc = self.lib.lvg_create_multi(self._cp.ptr, device_mask, C.byref(h))
        else:
            rc = self.lib.lvg_create(self._cp.ptr, device, C.byref(h))
        if rc != 0:
            raise LvgError(f"lvg_create failed ({rc}): {self.lib.lvg_last_error(None).decode()}")
        self.h = h

    def nb_devices(self) -> int:
        return self.lib.lvg_nb_devices(self.h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.lvg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise LvgError(f"{what} failed ({rc}): {self.lib.lvg_last_error(self.h).decode()}")

    def solve_layers(self, layers: abi.Layers, opts=None, pops=None):
        """Batched calc_molecular_populations over host buffers -> (pops [L,N], status)."""
        o = opts if opts is not None else abi.default_opts()
        cl = layers.to_c()
        out = np.zeros((layers.nb_lay, self.N)) if pops is None else np.array(pops, dtype=np.float64, copy=True)
        st = np.zeros(layers.nb_lay, dtype=abi.STATUS_DTYPE)
        rc = self.lib.lvg_solve_layers(self.h, cl.ptr, abi.dptr(out), C.byref(o), st.ctypes.data_as(C.c_void_p))
        self._check(rc, "lvg_solve_layers")
        return out, st

    def solve_chains(self, layers: abi.Layers, chain_off, opts=None):
        """Independent clouds, each a warm chain (layers [chain_off[c], chain_off[c+1])),
        in one launch -> (pops [L,N], status). opts.init must be LVG_INIT_WARM_CHAIN."""
        o = opts if opts is not None else abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN)
        cl = layers.to_c()
        off = np.ascontiguousarray(chain_off, dtype=np.int32)
        out = np.zeros((layers.nb_lay, self.N))
        st = np.zeros(layers.nb_lay, dtype=abi.STATUS_DTYPE)
        rc = self.lib.lvg_solve_chains(self.h, cl.ptr, len(off) - 1, off.ctypes.data_as(C.POINTER(C.c_int)),
                                       abi.dptr(out), C.byref(o), st.ctypes.data_as(C.c_void_p))
        self._check(rc, "lvg_solve_chains")
        return out, st

    def solve_chains_device(self, nb_lay: int, soa_ptr: int, chain_off, pops_ptr: int, status_ptr: int,
                            opts=None, stream_ptr: int = 0):
        """Device-resident warm chains; chain_off is a host int array [nb_chain + 1]."""
        o = opts if opts is not None else abi.default_opts(init=abi.LVG_INIT_WARM_CHAIN)
        off = np.ascontiguousarray(chain_off, dtype=np.int32)
        rc = self.lib.lvg_solve_chains_device(self.h, nb_lay, C.c_void_p(soa_ptr), len(off) - 1,
                                              off.ctypes.data_as(C.POINTER(C.c_int)), C.c_void_p(pops_ptr),
                                              C.byref(o), C.c_void_p(status_ptr),
                                              C.c_void_p(stream_ptr) if stream_ptr else None)
        self._check(rc, "lvg_solve_chains_device")

    def soa_rows(self) -> int:
        return self.lib.lvg_layer_soa_rows(self.h)

    def solve_layers_device(self, nb_lay: int, soa_ptr: int, pops_ptr: int, status_ptr: int, opts=None,
                            stream_ptr: int = 0):
        """Device-resident variant: raw device pointers (e.g. torch tensor.data_ptr())."""
        o = opts if opts is not None else abi.default_opts()
        rc = self.lib.lvg_solve_layers_device(self.h, nb_lay, C.c_void_p(soa_ptr), C.c_void_p(pops_ptr),
                                              C.byref(o), C.c_void_p(status_ptr),
                                              C.c_void_p(stream_ptr) if stream_ptr else None)
        self._check(rc, "lvg_solve_layers_device")

    def last_kernel_time(self):
        ms = C.c_double()
        n = C.c_int()
        self._check(self.lib.lvg_last_kernel_time(self.h, C.byref(ms), C.byref(n)), "lvg_last_kernel_time")
        return ms.value, n.value

    def set_tuning(self, spec: str = ""):
        """lvg_set_tuning: "key=value,..." (include/lvg_amd.h); never changes a result."""
        self._check(self.lib.lvg_set_tuning(self.h, spec.encode()), "lvg_set_tuning")

    def last_coll_time(self):
        """Milliseconds of the collision-operator kernel of the last solve (0: not run)."""
        ms = C.c_double()
        self._check(self.lib.lvg_last_coll_time(self.h, C.byref(ms)), "lvg_last_coll_time")
        return ms.value

    def last_kernel_kind(self):
        """The solve kernel of the last solve: 0 block (256 threads), 1 wave, 2 block (512
        threads, underfilled launches), 3 block (768 threads, N > 256)."""
        k = C.c_int()
        self._check(self.lib.lvg_last_kernel_kind(self.h, C.byref(k)), "lvg_last_kernel_kind")
        return k.value

    def debug_calc_new_pop(self, layers: abi.Layers, layer: int, pop_in, overlap: int = 0):
        cl = layers.to_c()
        pin = np.ascontiguousarray(pop_in, dtype=np.float64)
        M = np.zeros((self.N, self.N)); df = np.zeros(self.N); pout = np.zeros(self.N); e = C.c_double()
        rc = self.lib.lvg_debug_calc_new_pop(self.h, cl.ptr, layer, abi.dptr(pin), overlap, abi.dptr(M),
                                             abi.dptr(df), abi.dptr(pout), C.byref(e))
        self._check(rc, "lvg_debug_calc_new_pop")
        return M, df, pout, e.value

    def boundary_layer_populations(self, layers: abi.Layers):
        cl = layers.to_c()
        out = np.zeros((layers.nb_lay, self.N))
        self._check(self.lib.lvg_boundary_layer_populations(self.h, cl.ptr, abi.dptr(out)),
                    "lvg_boundary_layer_populations")
        return out

    def find_transitions(self, layers: abi.Layers, geo: "abi.Geometry", pops, opts=None, max_out: int = 256):
        """transition_data_container::find on the device -> (records, inv, gain, exc_temp):
        records is a TRANSITION_DTYPE array in the reference's list order, the per-layer
        arrays are [n, nb_lay]."""
        o = opts if opts is not None else abi.find_opts()
        cl = layers.to_c()
        cg = geo.to_c()
        p = np.ascontiguousarray(pops, dtype=np.float64)
        nl = layers.nb_lay
        while True:
            out = np.zeros(max_out, dtype=abi.TRANSITION_DTYPE)
            inv = np.zeros((max_out, nl)); gain = np.zeros((max_out, nl)); exc = np.zeros((max_out, nl))
            n = C.c_int()
            rc = self.lib.lvg_find_transitions(self.h, cl.ptr, C.byref(cg), abi.dptr(p), C.byref(o), max_out,
                                               C.byref(n), out.ctypes.data_as(C.c_void_p), abi.dptr(inv),
                                               abi.dptr(gain), abi.dptr(exc))
            self._check(rc, "lvg_find_transitions")
            if n.value <= max_out:
                k = n.value
                return out[:k].copy(), inv[:k].copy(), gain[:k].copy(), exc[:k].copy()
            max_out = n.value

    def lim_luminosity(self, layers: abi.Layers, geo: "abi.Geometry", pops, up, low, layer_pops: int = 0):
        """lim_luminosity_lvg on the device -> dict(lum [T], lum_arr, emiss, pump_rate, pump_eff,
        loss_rate [T, nb_lay])."""
        return _lim_lum_call(self.lib.lvg_lim_luminosity, lambda rc: self._check(rc, "lvg_lim_luminosity"),
                             self.h, layers, geo, pops, up, low, layer_pops)


def _lim_lum_call(fn, check, first, layers, geo, pops, up, low, layer_pops):
    cl, cg = layers.to_c(), geo.to_c()
    p = np.ascontiguousarray(pops, dtype=np.float64)
    u = np.ascontiguousarray(up, dtype=np.int32)
    lo = np.ascontiguousarray(low, dtype=np.int32)
    T, nl = len(u), layers.nb_lay
    out = {"lum": np.zeros(T)}
    for k in ("lum_arr", "emiss", "pump_rate", "pump_eff", "loss_rate"):
        out[k] = np.zeros((T, nl))
    rc = fn(first, cl.ptr, C.byref(cg), abi.dptr(p), T, abi.iptr(u), abi.iptr(lo), int(layer_pops), abi.dptr(out["lum"]),
            abi.dptr(out["lum_arr"]), abi.dptr(out["emiss"]), abi.dptr(out["pump_rate"]), abi.dptr(out["pump_eff"]),
            abi.dptr(out["loss_rate"]))
    check(rc)
    return out

