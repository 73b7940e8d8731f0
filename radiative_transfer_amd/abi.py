"""ctypes mirror of include/lvg_amd.h plus the numpy-backed description objects.

The C ABI takes plain pointers; this module owns the numpy arrays behind them
and builds the struct tree (``lvg_problem`` -> molecule / collisions / dust /
escape tables) and the layer SoA (``lvg_layers``). It carries no solver logic.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

# ---- enums (lvg_amd.h) ------------------------------------------------------
LVG_OK = 0
LVG_SP_HE, LVG_SP_PH2, LVG_SP_OH2, LVG_SP_H, LVG_SP_E = range(5)
LVG_COLL_GENERIC, LVG_COLL_CH3OH, LVG_COLL_H2O, LVG_COLL_OH, LVG_COLL_OH_HF = range(5)
LVG_INIT_BOUNDARY_LAYER, LVG_INIT_GIVEN, LVG_INIT_WARM_CHAIN = range(3)

LAYER_FIELDS = ("temp_n", "temp_el", "el_conc", "h_conc", "ph2_conc", "oh2_conc",
                "he_conc", "mol_conc", "vel_turb", "vel_grad")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class c_molecule(C.Structure):
    _fields_ = [("nb_lev", C.c_int), ("mass", C.c_double), ("energy", _dp), ("g", _ip),
                ("v", _ip), ("j", _dp), ("einst", _dp)]


class c_coll_table(C.Structure):
    _fields_ = [("nb_lev", C.c_int), ("jmax", C.c_int), ("tgrid", _dp), ("coeff", _dp),
                ("species", C.c_int)]


class c_collisions(C.Structure):
    _fields_ = [("rule", C.c_int), ("nb_neutral", C.c_int), ("nb_electron", C.c_int),
                ("tables", C.POINTER(c_coll_table))]


class c_dust_component(C.Structure):
    _fields_ = [("nb_en", C.c_int), ("wvl_exp", C.c_double), ("energy", _dp), ("abs_coeff", _dp)]


class c_dust(C.Structure):
    _fields_ = [("nb_comp", C.c_int), ("comp", C.POINTER(c_dust_component))]


class c_esc_table(C.Structure):
    _fields_ = [("nb_d", C.c_int), ("nb_g", C.c_int), ("delta", _dp), ("gamma", _dp), ("p", _dp)]


class c_overlap_table(C.Structure):
    _fields_ = [("nb_d", C.c_int), ("nb_dx", C.c_int), ("nb_gr", C.c_int), ("nb_g", C.c_int),
                ("log10_delta", _dp), ("dx", _dp), ("gratio", _dp), ("gamma", _dp), ("p", _dp)]


class c_problem(C.Structure):
    _fields_ = [("mol", C.POINTER(c_molecule)), ("coll", C.POINTER(c_collisions)),
                ("dust", C.POINTER(c_dust)), ("esc", C.POINTER(c_esc_table)),
                ("overlap1", C.POINTER(c_overlap_table)), ("overlap2", C.POINTER(c_overlap_table))]


class c_layers(C.Structure):
    _fields_ = [("nb_lay", C.c_int)] + [(f, _dp) for f in LAYER_FIELDS] + [("dust_conc", _dp)]


class c_solve_opts(C.Structure):
    _fields_ = [("min_error", C.c_double), ("max_iter_acc", C.c_int), ("max_iter_plain", C.c_int),
                ("accel_start", C.c_int), ("accel_period", C.c_int), ("accel_nb", C.c_int),
                ("acceleration", C.c_int), ("allow_plain_retry", C.c_int), ("init", C.c_int),
                ("line_overlap", C.c_int)]


class c_layer_status(C.Structure):
    _fields_ = [("converged", C.c_int), ("iterations", C.c_int), ("used_plain_retry", C.c_int),
                ("reserved", C.c_int), ("eq_error", C.c_double), ("rel_error", C.c_double),
                ("pop_error", C.c_double)]


STATUS_DTYPE = np.dtype([("converged", np.int32), ("iterations", np.int32),
                         ("used_plain_retry", np.int32), ("reserved", np.int32),
                         ("eq_error", np.float64), ("rel_error", np.float64),
                         ("pop_error", np.float64)])
assert STATUS_DTYPE.itemsize == C.sizeof(c_layer_status)


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# ---- description objects (mirror the reference's object graph) ---------------

@dataclass
class Molecule:
    """energy_diagram + einstein_coeff (spectroscopy.h:69-87, :179-190)."""
    name: str
    mass: float
    energy: np.ndarray           # [N] cm^-1
    g: np.ndarray                # [N] int
    einst: np.ndarray            # [N,N]; einst[i,j] = rate i->j
    v: Optional[np.ndarray] = None
    j: Optional[np.ndarray] = None
    spin: float = 0.5

    @property
    def nb_lev(self) -> int:
        return int(self.energy.shape[0])


@dataclass
class CollTable:
    """collision_data (coll_rates.h:12-41): coeff[imax, jmax], imax = n(n-1)/2."""
    nb_lev: int
    tgrid: np.ndarray
    coeff: np.ndarray
    species: int = 0
    name: str = ""


@dataclass
class Collisions:
    rule: int
    neutral: List[CollTable]
    electron: List[CollTable] = field(default_factory=list)


@dataclass
class DustComponent:
    energy: np.ndarray
    abs_coeff: np.ndarray
    wvl_exp: float


@dataclass
class EscTable:
    delta: np.ndarray
    gamma: np.ndarray
    p: np.ndarray        # [nb_d, nb_g]


@dataclass
class OverlapTable:
    log10_delta: np.ndarray
    dx: np.ndarray
    gratio: np.ndarray
    gamma: np.ndarray
    p: np.ndarray        # [nb_d*nb_dx, nb_gr*nb_g]


@dataclass
class Problem:
    mol: Molecule
    coll: Collisions
    dust: List[DustComponent]
    esc: EscTable
    overlap1: Optional[OverlapTable] = None
    overlap2: Optional[OverlapTable] = None

    def to_c(self) -> "CProblem":
        return CProblem(self)


class CProblem:
    """Keeps every numpy buffer alive while the C structs point into them."""

    def __init__(self, P: Problem):
        self._keep = []
        m = P.mol
        N = m.nb_lev
        k = self._keep
        e = _f64(m.energy); g = np.ascontiguousarray(m.g, dtype=np.int32)
        v = np.ascontiguousarray(m.v if m.v is not None else np.zeros(N), dtype=np.int32)
        jj = _f64(m.j if m.j is not None else np.zeros(N))
        A = _f64(m.einst).reshape(N * N)
        k += [e, g, v, jj, A]
        self.mol = c_molecule(N, float(m.mass), dptr(e), iptr(g), iptr(v), dptr(jj), dptr(A))

        tabs = list(P.coll.neutral) + list(P.coll.electron)
        self.tables = (c_coll_table * max(1, len(tabs)))()
        for i, t in enumerate(tabs):
            tg = _f64(t.tgrid); cf = _f64(t.coeff).reshape(-1)
            k += [tg, cf]
            assert cf.size == t.nb_lev * (t.nb_lev - 1) // 2 * tg.size, "coeff shape"
            self.tables[i] = c_coll_table(int(t.nb_lev), int(tg.size), dptr(tg), dptr(cf), int(t.species))
        self.coll = c_collisions(int(P.coll.rule), len(P.coll.neutral), len(P.coll.electron), self.tables)

        self.dcomp = (c_dust_component * max(1, len(P.dust)))()
        for i, d in enumerate(P.dust):
            de = _f64(d.energy); da = _f64(d.abs_coeff)
            k += [de, da]
            self.dcomp[i] = c_dust_component(int(de.size), float(d.wvl_exp), dptr(de), dptr(da))
        self.dust = c_dust(len(P.dust), self.dcomp)

        ed, eg, ep = _f64(P.esc.delta), _f64(P.esc.gamma), _f64(P.esc.p).reshape(-1)
        k += [ed, eg, ep]
        self.esc = c_esc_table(int(ed.size), int(eg.size), dptr(ed), dptr(eg), dptr(ep))

        self.ov = []
        for t in (P.overlap1, P.overlap2):
            if t is None:
                self.ov.append(None)
                continue
            a = [_f64(t.log10_delta), _f64(t.dx), _f64(t.gratio), _f64(t.gamma), _f64(t.p).reshape(-1)]
            k += a
            self.ov.append(c_overlap_table(a[0].size, a[1].size, a[2].size, a[3].size,
                                           *[dptr(x) for x in a]))
        self.prob = c_problem(C.pointer(self.mol), C.pointer(self.coll), C.pointer(self.dust),
                              C.pointer(self.esc),
                              C.pointer(self.ov[0]) if self.ov[0] is not None else None,
                              C.pointer(self.ov[1]) if self.ov[1] is not None else None)

    @property
    def ptr(self):
        return C.byref(self.prob)


@dataclass
class Layers:
    """cloud_layer fields read by the solver (cloud_data.h:27-33), as SoA."""
    temp_n: np.ndarray
    temp_el: np.ndarray
    el_conc: np.ndarray
    h_conc: np.ndarray
    ph2_conc: np.ndarray
    oh2_conc: np.ndarray
    he_conc: np.ndarray
    mol_conc: np.ndarray
    vel_turb: np.ndarray
    vel_grad: np.ndarray
    dust_conc: np.ndarray        # [nb_lay, nb_comp]

    @property
    def nb_lay(self) -> int:
        return int(self.temp_n.shape[0])

    def subset(self, idx) -> "Layers":
        return Layers(**{f: np.ascontiguousarray(getattr(self, f)[idx]) for f in LAYER_FIELDS + ("dust_conc",)})

    def soa(self) -> np.ndarray:
        """[10 + nb_comp, nb_lay] fp64 in lvg_layers field order (lvg_solve_layers_device)."""
        rows = [getattr(self, f) for f in LAYER_FIELDS]
        dc = np.atleast_2d(self.dust_conc)
        rows += [dc[:, c] for c in range(dc.shape[1])]
        return np.ascontiguousarray(np.stack(rows), dtype=np.float64)

    def to_c(self) -> "CLayers":
        return CLayers(self)


class CLayers:
    def __init__(self, L: Layers):
        self._keep = [_f64(getattr(L, f)) for f in LAYER_FIELDS]
        dc = _f64(L.dust_conc).reshape(-1)
        self._keep.append(dc)
        self.s = c_layers(L.nb_lay, *[dptr(a) for a in self._keep])

    @property
    def ptr(self):
        return C.byref(self.s)


# ---- post-processing (transition_data_container::find) ---------------------------------
NB_ASPECT = 37
NB_FREQ = 300


class c_cloud_geometry(C.Structure):
    _fields_ = [("dz", _dp), ("vel_n", _dp), ("height", C.c_double)]


class c_find_opts(C.Structure):
    _fields_ = [("rel_error", C.c_double), ("min_optical_depth", C.c_double), ("velocity_shift", C.c_double),
                ("delta_aspect_ratio", C.c_double), ("h2o22_up", C.c_int), ("h2o22_low", C.c_int)]


TRANSITION_DTYPE = np.dtype([("up", np.int32), ("low", np.int32), ("lay_nb_hg", np.int32), ("reserved", np.int32),
                             ("energy", np.float64), ("inv", np.float64), ("gain", np.float64),
                             ("tau_eff", np.float64), ("tau_max", np.float64),
                             ("tau_vs_aspect_ratio", np.float64, (NB_ASPECT,)),
                             ("tau_vs_frequency", np.float64, (NB_FREQ,))])


def find_opts(**kw) -> c_find_opts:
    o = c_find_opts(1e-5, 0.01, 5e5, 0.25, -1, -1)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


@dataclass
class Geometry:
    """cloud_layer::dz / vel_n and cloud_data::get_height() (cloud_data.h:27-29, .cpp:106)."""
    dz: np.ndarray
    vel_n: np.ndarray
    height: float

    def to_c(self):
        self._dz = np.ascontiguousarray(self.dz, dtype=np.float64)
        self._vel = np.ascontiguousarray(self.vel_n, dtype=np.float64)
        return c_cloud_geometry(dptr(self._dz), dptr(self._vel), float(self.height))


def default_opts(**kw) -> c_solve_opts:
    o = c_solve_opts(1e-5, 150, 15000, 40, 5, 5, 1, 1, LVG_INIT_BOUNDARY_LAYER, 0)
    for k, v in kw.items():
        setattr(o, k, v)
    return o
