"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It checks the product (motionplanningtoolkit_amd) and is never the
thing measured or shipped.  See mpt_oracle.h for what is restated and how the
oracle is pinned (parity against the reference itself is unpinned: the
reference ships no tests and cannot be built here).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmpt_oracle.so")
_lib = None

D = C.c_double
I32 = C.c_int32
I64 = C.c_int64
U64 = C.c_uint64
P = C.c_void_p


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def build_native(out_dir: str) -> str:
    """The same restatement compiled for the host it runs on (-O3 -march=native): bench.py's
    CPU-baseline leg builds it on the GPU box's own cores.  Returns the library path."""
    subprocess.run(["make", "-s", "-C", _HERE, f"OUT={out_dir}", "OPT=-O3 -march=native"], check=True)
    return os.path.join(out_dir, "libmpt_oracle.so")


def lib(path: str | None = None):
    """Load the oracle library (the portable -O3 build by default; `path` loads another
    build of the same source, e.g. build_native's, and replaces the loaded one)."""
    global _lib
    if path is not None and (_lib is None or _lib._name != path):
        _lib = None
    if _lib is None:
        if path is None and (not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "mpt_oracle.c")
        )):
            build()
        L = C.CDLL(path or _LIB_PATH)
        sig = {
            "orc_quat_to_rot": (None, [P, P]),
            "orc_relative_transform": (None, [P, P, P, P, P, P]),
            "orc_tri_intersect": (C.c_int, [P, P]),
            "orc_tri_intersect_RT": (C.c_int, [P, P, P, P]),
            "orc_collide_unit": (C.c_int, [P, I64, P, P, I64, P]),
            "orc_collide_batch": (None, [P, I64, P, P, P, I32, P, P, I64, P]),
            "orc_bvh_build": (P, [P, I64]),
            "orc_bvh_free": (None, [P]),
            "orc_collide_unit_bvh": (C.c_int, [P, P, P, I64, P, P]),
            "orc_collide_batch_bvh": (None, [P, P, P, P, I32, P, P, I64, P, C.c_int]),
            "orc_l2": (D, [P, P, I32]),
            "orc_knn": (None, [P, P, I64, I32, P, I64, I32, P, P]),
            "orc_radius": (I64, [P, P, I64, I32, P, I64, D, I32, P, P, P, I64]),
            "orc_kdtree_build": (P, [P, I64, I32]),
            "orc_kdtree_free": (None, [P]),
            "orc_kdtree_knn": (None, [P, P, I64, I32, P, P, C.c_int]),
            "orc_glibc_srand": (None, [P, C.c_uint32]),
            "orc_glibc_rand_next": (I32, [P]),
            "orc_minstd_seed": (None, [P, U64]),
            "orc_minstd_next": (U64, [P]),
            "orc_uniform_real": (D, [P, D, D]),
            "orc_engine_uniform": (D, [U64, U64, D, D]),
            "orc_omni_get_poses": (I32, [P, P, D, P, I32]),
            "orc_blimp_do_step": (None, [P, P, D, D, D, D, P]),
            "orc_blimp_get_poses": (I32, [P, P, P, D, D, P, I32]),
            "orc_snake_do_step": (None, [P, P, D, D, D, P]),
            "orc_snake_get_poses": (I32, [P, P, P, D, D, P, I32]),
            "orc_cr_sin": (D, [D]),
            "orc_cr_cos": (D, [D]),
            "orc_cr_tan": (D, [D]),
            "orc_blimp_do_step_cr": (None, [P, P, D, D, D, D, P]),
            "orc_blimp_get_poses_cr": (I32, [P, P, P, D, D, P, I32]),
            "orc_snake_do_step_cr": (None, [P, P, D, D, D, P]),
            "orc_snake_get_poses_cr": (I32, [P, P, P, D, D, P, I32]),
            "orc_rrt_run": (I64, [I32, P, I32, P, P, P, P, D, D, P, I64, P, P, I64, I64, I64, P, P, P, P]),
            "orc_engine_step": (I64, [I32, P, I32, P, D, D, U64, U64, I32, P, P, P, I64, P, P, I64, I64, P, P, C.c_int, C.c_int]),
            "orc_rrt_seq_rebuild": (I64, [I32, P, I32, P, D, D, U64, U64, I64, D, P, P, P, I64, P, P, I64, I64, P, P]),
            "orc_prm_build": (I64, [P, P, P, I64, P, I64, I32, I32, D, P, P, I64, P]),
            "orc_tri_distance": (D, [P, P]),
            "orc_grid_discretization": (I64, [P, P, P, I64, P, P, I32, P, I64]),
            "orc_prmlite_edges": (None, [P, P, P, I64, P, I64, D, P, C.c_int]),
            "orc_self_collide_batch": (None, [P, P, I32, P, P, I64, P]),
            "orc_prm_radius": (I64, [P, P, P, I64, P, I64, I32, D, D, P, P, I64, P, C.c_int]),
            "orc_distance_unit": (D, [P, I64, P, P, I64, P]),
            "orc_distance_batch": (None, [P, I64, P, P, P, I32, P, P, I64, P, C.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def quat_to_rot(q) -> np.ndarray:
    q = _f64(q)
    R = np.zeros(9)
    lib().orc_quat_to_rot(_p(q), _p(R))
    return R


def env_tf_from_location(loc) -> np.ndarray:
    """parseTransform('x y z qw qx qy qz') -> R (9, row-major) + T (3)."""
    loc = _f64(loc)
    return np.concatenate([quat_to_rot(loc[3:7]), loc[:3]])


def tri_intersect(P, Q) -> bool:
    return bool(lib().orc_tri_intersect(_p(_f64(P)), _p(_f64(Q))))


def collide_batch(env_tris, env_tf, link_tris: list, poses, edge_offsets) -> np.ndarray:
    """All-pairs FCL verdicts. poses [sumP][L][12], edge_offsets [E+1]."""
    env_tris = _f64(env_tris).reshape(-1, 9)
    agent = _f64(np.concatenate([np.asarray(t, np.float64).reshape(-1, 9) for t in link_tris]))
    off = np.zeros(len(link_tris) + 1, np.int64)
    off[1:] = np.cumsum([np.asarray(t).reshape(-1, 9).shape[0] for t in link_tris])
    poses = _f64(poses)
    eo = np.ascontiguousarray(edge_offsets, np.int64)
    E = len(eo) - 1
    out = np.zeros(E, np.uint8)
    lib().orc_collide_batch(_p(env_tris), env_tris.shape[0], _p(_f64(env_tf)), _p(agent), _p(off),
                            len(link_tris), _p(poses), _p(eo), E, _p(out))
    return out


def prm_radius(bvh: BVH, env_tf, agent_tris, states, r2: float, cc_dt: float, nthreads=8):
    """orc_prm_radius: (edges [E][2] = (i, j), verdict [E], comp [n])."""
    st = _f64(states)
    n, dim = st.shape
    at = _f64(agent_tris).reshape(-1, 9)
    E = lib().orc_prm_radius(bvh.ptr, _p(_f64(env_tf)), _p(at), at.shape[0], _p(st), n, dim, r2, cc_dt, None, None, 0,
                             None, nthreads)
    edges = np.zeros((max(E, 1), 2), np.int32)
    verdict = np.zeros(max(E, 1), np.uint8)
    comp = np.zeros(max(n, 1), np.int32)
    lib().orc_prm_radius(bvh.ptr, _p(_f64(env_tf)), _p(at), at.shape[0], _p(st), n, dim, r2, cc_dt, _p(edges),
                         _p(verdict), E, _p(comp), nthreads)
    return edges[:E], verdict[:E], comp[:n]


def self_collide_batch(link_tris: list, poses, edge_offsets) -> np.ndarray:
    """Link-vs-link verdicts per edge (checkSelfCollision branch)."""
    agent = _f64(np.concatenate([np.asarray(t, np.float64).reshape(-1, 9) for t in link_tris]))
    off = np.zeros(len(link_tris) + 1, np.int64)
    off[1:] = np.cumsum([np.asarray(t).reshape(-1, 9).shape[0] for t in link_tris])
    poses = _f64(poses)
    eo = np.ascontiguousarray(edge_offsets, np.int64)
    E = len(eo) - 1
    out = np.zeros(E, np.uint8)
    lib().orc_self_collide_batch(_p(agent), _p(off), len(link_tris), _p(poses), _p(eo), E, _p(out))
    return out


def prmlite_edges(bvh: BVH, env_tf, agent_tris, verts, step=0.1, nthreads=8) -> np.ndarray:
    v = _f64(verts).reshape(-1, 12)
    V = v.shape[0]
    at = _f64(agent_tris).reshape(-1, 9)
    out = np.zeros(max(V * (V - 1) // 2, 0), np.uint8)
    lib().orc_prmlite_edges(bvh.ptr, _p(_f64(env_tf)), _p(at), at.shape[0], _p(v), V, step, _p(out), nthreads)
    return out


def grid_discretization(bvh: BVH, env_tf, agent_tris, bounds, sizes, n_rot) -> np.ndarray:
    at = _f64(agent_tris).reshape(-1, 9)
    b, s = _f64(bounds).ravel(), _f64(sizes)
    n = lib().orc_grid_discretization(bvh.ptr, _p(_f64(env_tf)), _p(at), at.shape[0], _p(b), _p(s), n_rot, None, 0)
    out = np.zeros(n, np.uint8)
    lib().orc_grid_discretization(bvh.ptr, _p(_f64(env_tf)), _p(at), at.shape[0], _p(b), _p(s), n_rot, _p(out), n)
    return out.astype(bool)


def tri_distance(S, T) -> float:
    """FCL triDistance (T already in S's frame) with the box-gated overlap answer."""
    return float(lib().orc_tri_distance(_p(_f64(S)), _p(_f64(T))))


def distance_batch(env_tris, env_tf, link_tris: list, poses, edge_offsets, nthreads=1) -> np.ndarray:
    """Per-edge minimum mesh-vs-mesh distance (DBL_MAX for an edge without poses)."""
    env_tris = _f64(env_tris).reshape(-1, 9)
    agent = _f64(np.concatenate([np.asarray(t, np.float64).reshape(-1, 9) for t in link_tris]))
    off = np.zeros(len(link_tris) + 1, np.int64)
    off[1:] = np.cumsum([np.asarray(t).reshape(-1, 9).shape[0] for t in link_tris])
    poses = _f64(poses)
    eo = np.ascontiguousarray(edge_offsets, np.int64)
    E = len(eo) - 1
    out = np.zeros(E)
    lib().orc_distance_batch(_p(env_tris), env_tris.shape[0], _p(_f64(env_tf)), _p(agent), _p(off),
                             len(link_tris), _p(poses), _p(eo), E, _p(out), nthreads)
    return out


class BVH:
    def __init__(self, tris):
        self._tris = _f64(tris).reshape(-1, 9)
        self.ptr = lib().orc_bvh_build(_p(self._tris), self._tris.shape[0])

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().orc_bvh_free(self.ptr)
            self.ptr = None


def collide_batch_bvh(bvh: BVH, env_tf, link_tris: list, poses, edge_offsets, nthreads=1) -> np.ndarray:
    agent = _f64(np.concatenate([np.asarray(t, np.float64).reshape(-1, 9) for t in link_tris]))
    off = np.zeros(len(link_tris) + 1, np.int64)
    off[1:] = np.cumsum([np.asarray(t).reshape(-1, 9).shape[0] for t in link_tris])
    poses = _f64(poses)
    eo = np.ascontiguousarray(edge_offsets, np.int64)
    E = len(eo) - 1
    out = np.zeros(E, np.uint8)
    lib().orc_collide_batch_bvh(bvh.ptr, _p(_f64(env_tf)), _p(agent), _p(off), len(link_tris),
                                _p(poses), _p(eo), E, _p(out), nthreads)
    return out


def l2(a, b) -> float:
    a = _f64(a)
    b = _f64(b)
    return lib().orc_l2(_p(a), _p(b), a.shape[0])


def knn(pts, q, k, removed=None):
    pts = _f64(pts)
    n, d = pts.shape
    q = _f64(q).reshape(-1, d)
    ids = np.zeros((q.shape[0], k), np.int32)
    d2 = np.zeros((q.shape[0], k), np.float64)
    rem = None if removed is None else np.ascontiguousarray(removed, np.uint8)
    lib().orc_knn(_p(pts), _p(rem), n, d, _p(q), q.shape[0], k, _p(ids), _p(d2))
    return ids, d2


def radius(pts, q, r2, max_nb=-1, removed=None):
    pts = _f64(pts)
    n, d = pts.shape
    q = _f64(q).reshape(-1, d)
    nq = q.shape[0]
    off = np.zeros(nq + 1, np.int64)
    rem = None if removed is None else np.ascontiguousarray(removed, np.uint8)
    total = lib().orc_radius(_p(pts), _p(rem), n, d, _p(q), nq, r2, max_nb, _p(off), None, None, 0)
    ids = np.zeros(max(total, 1), np.int32)
    d2 = np.zeros(max(total, 1), np.float64)
    lib().orc_radius(_p(pts), _p(rem), n, d, _p(q), nq, r2, max_nb, _p(off), _p(ids), _p(d2), total)
    return off, ids[:total], d2[:total]


class KDTree:
    def __init__(self, pts):
        self._pts = _f64(pts)
        self.d = self._pts.shape[1]
        self.ptr = lib().orc_kdtree_build(_p(self._pts), self._pts.shape[0], self.d)

    def knn(self, q, k, nthreads=1):
        q = _f64(q).reshape(-1, self.d)
        ids = np.zeros((q.shape[0], k), np.int32)
        d2 = np.zeros((q.shape[0], k), np.float64)
        lib().orc_kdtree_knn(self.ptr, _p(q), q.shape[0], k, _p(ids), _p(d2), nthreads)
        return ids, d2

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().orc_kdtree_free(self.ptr)
            self.ptr = None


class GlibcRand(C.Structure):
    _fields_ = [("r", C.c_int32 * 34), ("f", C.c_int32), ("b", C.c_int32)]

    def __init__(self, seed=1):
        super().__init__()
        lib().orc_glibc_srand(C.byref(self), seed)

    def next(self) -> int:
        return lib().orc_glibc_rand_next(C.byref(self))


class Minstd(C.Structure):
    _fields_ = [("x", C.c_uint64)]

    def __init__(self, seed=1):
        super().__init__()
        lib().orc_minstd_seed(C.byref(self), seed)

    def next(self) -> int:
        return lib().orc_minstd_next(C.byref(self))

    def uniform(self, a, b) -> float:
        return lib().orc_uniform_real(C.byref(self), a, b)


def engine_uniform(seed, counter, a, b) -> float:
    return lib().orc_engine_uniform(seed, counter, a, b)


def omni_get_poses(start, end, dt, maxP=4096):
    out = np.zeros((maxP, 12))
    P = lib().orc_omni_get_poses(_p(_f64(start)), _p(_f64(end)), dt, _p(out), maxP)
    return out[: min(P, maxP)]


# trig: "libm" = the host libm (the reference's std::sin / cos / tan: the sequential loops);
# "cr" = correctly rounded (the batched engine round's contract, orc_cr_sin / cos / tan)
def _sfx(trig):
    if trig not in ("libm", "cr"):
        raise ValueError(trig)
    return "_cr" if trig == "cr" else ""


def cr_sin(x) -> float:
    return lib().orc_cr_sin(float(x))


def cr_cos(x) -> float:
    return lib().orc_cr_cos(float(x))


def cr_tan(x) -> float:
    return lib().orc_cr_tan(float(x))


def blimp_do_step(prm, s, a, w, z, dt, trig="libm"):
    out = np.zeros(7)
    getattr(lib(), "orc_blimp_do_step" + _sfx(trig))(_p(_f64(prm)), _p(_f64(s)), a, w, z, dt, _p(out))
    return out


def blimp_get_poses(prm, start, awz, edge_dt, dt, maxP=4096, trig="libm"):
    out = np.zeros((maxP, 12))
    P = getattr(lib(), "orc_blimp_get_poses" + _sfx(trig))(_p(_f64(prm)), _p(_f64(start)), _p(_f64(awz)), edge_dt,
                                                           dt, _p(out), maxP)
    return out[: min(P, maxP)]


def snake_do_step(prm, s, a, w, dt, trig="libm"):
    s = _f64(s)
    out = np.zeros_like(s)
    getattr(lib(), "orc_snake_do_step" + _sfx(trig))(_p(_f64(prm)), _p(s), a, w, dt, _p(out))
    return out


def snake_get_poses(prm, start, aw, edge_dt, dt, maxP=64, trig="libm"):
    L = int(prm[0]) + 1
    out = np.zeros((maxP, L, 12))
    P = getattr(lib(), "orc_snake_get_poses" + _sfx(trig))(_p(_f64(prm)), _p(_f64(start)), _p(_f64(aw)), edge_dt, dt,
                                                           _p(out), maxP)
    return out[: min(P, maxP)]


def rrt_run(kind, prm, ranges, start, goal, thr, steer_dt, cc_dt, env_tris, env_tf, agent_tris,
            max_iters, max_nodes):
    ranges = _f64(ranges).reshape(-1, 2)
    d = ranges.shape[0]
    nodes = np.zeros((max_nodes, d))
    parents = np.zeros(max_nodes, np.int32)
    solved = C.c_int64(0)
    iters = C.c_int64(0)
    env_tris = _f64(env_tris).reshape(-1, 9)
    agent_tris = _f64(agent_tris).reshape(-1, 9)
    prm = _f64(prm if prm is not None else np.zeros(7))
    n = lib().orc_rrt_run(kind, _p(prm), d, _p(ranges), _p(_f64(start)), _p(_f64(goal)), _p(_f64(thr)),
                          steer_dt, cc_dt, _p(env_tris), env_tris.shape[0], _p(_f64(env_tf)),
                          _p(agent_tris), agent_tris.shape[0], max_iters, max_nodes,
                          _p(nodes), _p(parents), C.byref(solved), C.byref(iters))
    return nodes[:n], parents[:n], solved.value, iters.value


def engine_step(kind, prm, ranges, steer_dt, cc_dt, seed, ext_base, K, bvh: BVH, env_tf, agent_tris,
                nodes, parents, n_nodes, nthreads=1, use_kdtree=True):
    """Mutates nodes/parents in place; returns (new n_nodes, nn ids [K], verdicts [K])."""
    ranges = _f64(ranges).reshape(-1, 2)
    d = ranges.shape[0]
    assert nodes.dtype == np.float64 and nodes.flags.c_contiguous and nodes.shape[1] == d
    assert parents.dtype == np.int32
    agent_tris = _f64(agent_tris).reshape(-1, 9)
    nn = np.zeros(K, np.int32)
    verdict = np.zeros(K, np.uint8)
    prm = _f64(prm if prm is not None else np.zeros(7))
    n = lib().orc_engine_step(kind, _p(prm), d, _p(ranges), steer_dt, cc_dt, seed, ext_base, K, bvh.ptr,
                              _p(_f64(env_tf)), _p(agent_tris), agent_tris.shape[0], _p(nodes), _p(parents),
                              n_nodes, nodes.shape[0], _p(nn), _p(verdict), nthreads, 1 if use_kdtree else 0)
    return n, nn, verdict


def rrt_seq_rebuild(kind, prm, ranges, steer_dt, cc_dt, seed, ext_base, bvh: BVH, env_tf, agent_tris, nodes,
                    parents, n_nodes, max_ext, time_budget):
    """orc_rrt_seq_rebuild: the reference's one-extension-at-a-time loop with a kd-tree rebuild
    per insertion (FLANN 1.8.4 addPoints).  Mutates nodes/parents; returns (valid, tried, s)."""
    ranges = _f64(ranges).reshape(-1, 2)
    d = ranges.shape[0]
    assert nodes.dtype == np.float64 and nodes.flags.c_contiguous and nodes.shape[1] == d
    agent_tris = _f64(agent_tris).reshape(-1, 9)
    prm = _f64(prm if prm is not None else np.zeros(7))
    done, secs = C.c_int64(), C.c_double()
    valid = lib().orc_rrt_seq_rebuild(kind, _p(prm), d, _p(ranges), steer_dt, cc_dt, seed, ext_base, max_ext,
                                      time_budget, bvh.ptr, _p(_f64(env_tf)), _p(agent_tris), agent_tris.shape[0],
                                      _p(nodes), _p(parents), n_nodes, nodes.shape[0], C.byref(done), C.byref(secs))
    return valid, done.value, secs.value


def prm_build(bvh: BVH, env_tf, agent_tris, states, k=10, batch=1, cc_dt=0.1):
    """PRM roadmap over explicit omnidirectional milestones (orc_prm_build): returns
    (edges [E][2] = (target, source), costs [E], comp [n])."""
    states = _f64(states).reshape(-1, 3)
    n = states.shape[0]
    agent_tris = _f64(agent_tris).reshape(-1, 9)
    cap = max(1, n * k)
    edges = np.zeros((cap, 2), np.int32)
    costs = np.zeros(cap)
    comp = np.zeros(n, np.int32)
    ne = lib().orc_prm_build(bvh.ptr, _p(_f64(env_tf)), _p(agent_tris), agent_tris.shape[0], _p(states), n, k, batch,
                             cc_dt, _p(edges), _p(costs), cap, _p(comp))
    assert ne >= 0
    return edges[:ne], costs[:ne], comp
