"""Python face of libmpt.so: thin owners of the C-ABI handles (include/mpt.h).

Mirrors the reference's native seams for the RRT/PRM inner loop:

* :class:`Environment` / :class:`AgentMesh` -- StaticEnvironmentMeshHandler /
  SimpleAgentMeshHandler (utilities/meshhandler.hpp:16-183);
* :func:`collide_batch` -- MeshHandler::isInCollision for a batch of edges
  (utilities/meshhandler.hpp:187-243, via Map3D::safeEdge, workspaces/map3d.hpp:33-37);
* :class:`NearestNeighbors` -- FLANN_KDTreeWrapper (utilities/flannkdtreewrapper.hpp:8-125);
* :class:`RRTEngine` -- batched rounds of the RRT hot loop (planners/rrt.hpp:42-94).

Device work happens only inside libmpt; NumPy arrays are host staging, torch tensors
(optional) are accepted for the ``*_device`` entry points as device-memory plumbing.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from ._native import check, lib

AGENT_OMNI, AGENT_BLIMP, AGENT_SNAKE = 0, 1, 2


def _p(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(C.c_void_p)
    if hasattr(a, "data_ptr"):  # torch tensor on the device
        return C.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return C.c_void_p(a)
    raise TypeError(f"cannot pass {type(a)} as a pointer")


def _f64(a, shape=None) -> np.ndarray:
    x = np.ascontiguousarray(a, dtype=np.float64)
    return x.reshape(shape) if shape is not None else x


def _stream(stream):
    if stream is None:
        return None
    if hasattr(stream, "cuda_stream"):  # torch.cuda.Stream
        return C.c_void_p(stream.cuda_stream)
    return C.c_void_p(int(stream))


def init(device: int = 0) -> None:
    """mpt_init: select the device; fails unless it is a gfx950 (MI355X)."""
    check(lib().mpt_init(device), "mpt_init")


def synchronize() -> None:
    check(lib().mpt_device_synchronize(), "mpt_device_synchronize")


def transform_from_location(loc7) -> np.ndarray:
    """fcl_helpers::parseTransform('x y z qw qx qy qz') -> R (row-major) | T as 12 doubles."""
    loc = _f64(loc7, (7,))
    out = np.zeros(12)
    check(lib().mpt_transform_from_location(_p(loc), _p(out)), "mpt_transform_from_location")
    return out


class Environment:
    """Device-resident environment soup + BVH (StaticEnvironmentMeshHandler)."""

    def __init__(self, tris, tf12=None):
        self.tris = _f64(tris).reshape(-1, 9)
        self.tf = _f64(tf12 if tf12 is not None else np.r_[np.eye(3).ravel(), 0, 0, 0], (12,))
        h = C.c_void_p()
        check(lib().mpt_env_create(_p(self.tris), self.tris.shape[0], _p(self.tf), C.byref(h)), "mpt_env_create")
        self.handle = h

    def info(self) -> dict:
        out = np.zeros(3, np.int64)
        check(lib().mpt_env_info(self.handle, _p(out)), "mpt_env_info")
        return {"triangles": int(out[0]), "bvh_nodes": int(out[1]), "bvh_depth": int(out[2])}

    def close(self):
        if getattr(self, "handle", None):
            lib().mpt_env_destroy(self.handle)
            self.handle = None

    __del__ = close


class AgentMesh:
    """Device-resident agent link mesh (SimpleAgentMeshHandler)."""

    def __init__(self, tris):
        self.tris = _f64(tris).reshape(-1, 9)
        h = C.c_void_p()
        check(lib().mpt_agent_create(_p(self.tris), self.tris.shape[0], C.byref(h)), "mpt_agent_create")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            lib().mpt_agent_destroy(self.handle)
            self.handle = None

    __del__ = close


def _links(links: Sequence[AgentMesh]):
    arr = (C.c_void_p * len(links))(*[l.handle.value for l in links])
    return arr


def collide_batch(env: Environment, links: Sequence[AgentMesh], poses, edge_offsets, stream=None,
                  check_self: bool = False) -> np.ndarray:
    """Verdicts (1 = collision) for E edges; poses [sum P][L][12], edge_offsets [E+1].
    check_self: also link-vs-link contacts within a pose (isInCollision's checkSelfCollision)."""
    L = len(links)
    poses = _f64(poses).reshape(-1, L, 12)
    off = np.ascontiguousarray(edge_offsets, dtype=np.int64)
    E = off.shape[0] - 1
    out = np.zeros(max(E, 0), np.uint8)
    check(lib().mpt_collide_batch_ex(env.handle, _links(links), L, _p(poses), _p(off), E, int(check_self), _p(out),
                                     _stream(stream)), "mpt_collide_batch_ex")
    return out


def collide_batch_device(env: Environment, links: Sequence[AgentMesh], d_poses, d_offsets, E: int,
                         total_poses: int, d_verdict, stream=None) -> None:
    check(lib().mpt_collide_batch_device(env.handle, _links(links), len(links), _p(d_poses), _p(d_offsets), E,
                                         total_poses, _p(d_verdict), _stream(stream)), "mpt_collide_batch_device")


def distance_batch(env: Environment, links: Sequence[AgentMesh], poses, edge_offsets, stream=None) -> np.ndarray:
    """Minimum mesh-vs-mesh distance per edge (fcl::distance through defaultDistanceFunction,
    utilities/fcl_helpers.hpp:67-84): 0 = contact, DBL_MAX for an edge without poses."""
    L = len(links)
    poses = _f64(poses).reshape(-1, L, 12)
    off = np.ascontiguousarray(edge_offsets, dtype=np.int64)
    E = off.shape[0] - 1
    out = np.zeros(max(E, 0), np.float64)
    check(lib().mpt_distance_batch(env.handle, _links(links), L, _p(poses), _p(off), E, _p(out), _stream(stream)),
          "mpt_distance_batch")
    return out


def distance_batch_device(env: Environment, links: Sequence[AgentMesh], d_poses, d_offsets, E: int,
                          total_poses: int, d_dist, stream=None) -> None:
    check(lib().mpt_distance_batch_device(env.handle, _links(links), len(links), _p(d_poses), _p(d_offsets), E,
                                          total_poses, _p(d_dist), _stream(stream)), "mpt_distance_batch_device")


def prm_connect(env: Environment, agent: AgentMesh, kind: int, states, radius2: float, cc_dt: float) -> dict:
    """PRM roadmap with radius neighbours on the device (config 4, include/mpt.h mpt_prm_connect).
    Returns edges [E][2] = (i, j), verdict [E] (1 = in collision), comp [n], ms (stage times)."""
    st = _f64(states)
    n, dim = st.shape
    ne = C.c_int64()
    cap = max(64 * n, 1024)  # room for a mean of 64 earlier neighbours; re-run only beyond that
    while True:
        edges = np.zeros((cap, 2), np.int32)
        verdict = np.zeros(cap, np.uint8)
        comp = np.zeros(max(n, 1), np.int32)
        ms = np.zeros(4, np.float32)
        check(lib().mpt_prm_connect(env.handle, agent.handle, kind, _p(st), n, dim, radius2, cc_dt, cap, _p(edges),
                                    _p(verdict), C.byref(ne), _p(comp), _p(ms)), "mpt_prm_connect")
        E = ne.value
        if E <= cap:
            break
        cap = E
    return {"edges": edges[:E], "verdict": verdict[:E], "comp": comp[:n],
            "ms": dict(zip(["neighbours", "poses", "collision", "total"], ms.tolist()))}


def prm_stats(enable: bool) -> dict:
    """The sweep work counters of this thread's last prm_connect made with counters on; enable
    turns them on (or off) for later calls (diagnostics: an atomic per wave)."""
    out = np.zeros(8, np.uint64)
    check(lib().mpt_prm_stats(1 if enable else 0, _p(out), len(out)), "mpt_prm_stats")
    return dict(zip(["waves", "item_tests", "gate_tests", "sat_tests", "edges", "poses", "candidates",
                     "deferred_edges"], (int(x) for x in out)))


def prmlite_edges(env: Environment, agent: AgentMesh, vertices, step: float = 0.1) -> np.ndarray:
    """PRMLite::generateEdges on the device: collides [V(V-1)/2] over the pairs i < j (row-major)
    of vertices [V][12] (R | T)."""
    v = _f64(vertices).reshape(-1, 12)
    V = v.shape[0]
    out = np.zeros(max(V * (V - 1) // 2, 0), np.uint8)
    check(lib().mpt_prmlite_edges(env.handle, agent.handle, _p(v), V, step, _p(out), None), "mpt_prmlite_edges")
    return out


def prm_deferred_edges() -> np.ndarray:
    """The edge indices this thread's last prm_connect made with counters on (prm_stats(True))
    sent to the sweep's per-edge pass: the candidate pass's capped edges, then a full queue's."""
    n = C.c_int64(0)
    check(lib().mpt_prm_deferred_edges(None, 0, C.byref(n)), "mpt_prm_deferred_edges")
    out = np.zeros(n.value, np.int32)
    check(lib().mpt_prm_deferred_edges(_p(out), n.value, C.byref(n)), "mpt_prm_deferred_edges")
    return out


def set_sweep_queue_cap(max_candidates: int) -> None:
    """Test hook: cap the PRM sweep's candidate queue (0 restores the sized queue), so that the
    full-queue path (edges deferred to the per-edge sweep) runs on a small roadmap."""
    check(lib().mpt_set_sweep_queue_cap(int(max_candidates)), "mpt_set_sweep_queue_cap")


COLLIDE_MODES = {"split": 0, "fused": 1}


def set_collide_mode(mode: str) -> None:
    """Collision kernel structure: "split" (broad phase -> candidate pairs -> exact test,
    default) or "fused" (BVH walk with the exact test at the leaves).  Same verdicts."""
    check(lib().mpt_set_collide_mode(COLLIDE_MODES[mode]), "mpt_set_collide_mode")


def set_collide_stats(enable: bool) -> None:
    check(lib().mpt_set_stats(1 if enable else 0), "mpt_set_stats")


def last_collide_stats() -> dict:
    out = np.zeros(4, np.uint64)
    check(lib().mpt_last_collide_stats(_p(out)), "mpt_last_collide_stats")
    return {"units": int(out[0]), "clusters": int(out[1]), "node_visits": int(out[2]), "tri_tests": int(out[3])}


class NearestNeighbors:
    """FLANN_KDTreeWrapper on the device: exact, 1-based ids, squared L2 in FLANN order."""

    def __init__(self, dim: int, capacity: int = 1024):
        self.dim = dim
        h = C.c_void_p()
        check(lib().mpt_nn_create(dim, capacity, C.byref(h)), "mpt_nn_create")
        self.handle = h

    def append(self, pts) -> np.ndarray:
        pts = _f64(pts).reshape(-1, self.dim)
        ids = np.zeros(pts.shape[0], np.int32)
        check(lib().mpt_nn_append(self.handle, _p(pts), pts.shape[0], _p(ids)), "mpt_nn_append")
        return ids

    def set_index(self, mode: str) -> None:
        """'auto' | 'brute' | 'grid' (all exact, identical results)."""
        check(lib().mpt_nn_set_index(self.handle, {"auto": 0, "brute": 1, "grid": 2}[mode]), "mpt_nn_set_index")

    def remove(self, point_id: int) -> None:
        check(lib().mpt_nn_remove(self.handle, int(point_id)), "mpt_nn_remove")

    def __len__(self) -> int:
        n = C.c_int64()
        check(lib().mpt_nn_size(self.handle, C.byref(n)), "mpt_nn_size")
        return n.value

    def knn(self, q, k: int = 1, stream=None):
        q = _f64(q).reshape(-1, self.dim)
        ids = np.zeros((q.shape[0], k), np.int32)
        d2 = np.zeros((q.shape[0], k), np.float64)
        check(lib().mpt_nn_knn(self.handle, _p(q), q.shape[0], k, _p(ids), _p(d2), _stream(stream)), "mpt_nn_knn")
        return ids, d2

    def knn_device(self, d_q, nq: int, k: int, d_ids, d_d2, stream=None) -> None:
        check(lib().mpt_nn_knn_device(self.handle, _p(d_q), nq, k, _p(d_ids), _p(d_d2), _stream(stream)),
              "mpt_nn_knn_device")

    def radius(self, q, r2: float, max_nb: int = -1):
        """kNearestWithin: per query (offsets, ids, d2) with d2 < r2, sorted by (d2, id)."""
        q = _f64(q).reshape(-1, self.dim)
        nq = q.shape[0]
        off = np.zeros(nq + 1, np.int64)
        check(lib().mpt_nn_radius(self.handle, _p(q), nq, r2, max_nb, _p(off), None, None, 0, None), "mpt_nn_radius")
        total = int(off[-1])
        ids = np.zeros(max(total, 1), np.int32)
        d2 = np.zeros(max(total, 1), np.float64)
        check(lib().mpt_nn_radius(self.handle, _p(q), nq, r2, max_nb, _p(off), _p(ids), _p(d2), total, None),
              "mpt_nn_radius")
        return off, ids[:total], d2[:total]

    def close(self):
        if getattr(self, "handle", None):
            lib().mpt_nn_destroy(self.handle)
            self.handle = None

    __del__ = close


class RRTEngine:
    """Device-resident batched RRT (K extensions per round against the tree snapshot)."""

    def __init__(self, env: Environment, agent: AgentMesh, kind: int, prm, ranges, steer_dt: float, cc_dt: float,
                 capacity: int, seed: int = 0):
        self.env, self.agent = env, agent  # keep the handles alive
        self.ranges = _f64(ranges).reshape(-1, 2)
        self.dim = self.ranges.shape[0]
        prm_a = _f64(prm if prm is not None else np.zeros(7), (7,))
        h = C.c_void_p()
        check(lib().mpt_rrt_create(env.handle, agent.handle, kind, _p(prm_a), _p(self.ranges), self.dim, steer_dt,
                                   cc_dt, capacity, seed, C.byref(h)), "mpt_rrt_create")
        self.handle = h
        self.capacity = capacity

    def add_nodes(self, states, parents=None) -> None:
        s = _f64(states).reshape(-1, self.dim)
        par = None if parents is None else np.ascontiguousarray(parents, np.int32)
        check(lib().mpt_rrt_add_nodes(self.handle, _p(s), _p(par), s.shape[0]), "mpt_rrt_add_nodes")

    def set_size(self, n: int, stream=None) -> None:
        check(lib().mpt_rrt_set_size(self.handle, n, _stream(stream)), "mpt_rrt_set_size")

    def step(self, K: int, stream=None) -> None:
        check(lib().mpt_rrt_step(self.handle, K, _stream(stream)), "mpt_rrt_step")

    def counters(self) -> dict:
        c = np.zeros(8, np.uint64)
        check(lib().mpt_rrt_counters(self.handle, _p(c)), "mpt_rrt_counters")
        return {"rounds": int(c[0]), "checked": int(c[1]), "valid": int(c[2]), "nodes": int(c[3]),
                "capacity_drops": int(c[4]), "pose_overflow": int(c[5])}

    def read_tree(self, n: int):
        s = np.zeros((n, self.dim))
        p = np.zeros(n, np.int32)
        check(lib().mpt_rrt_read_tree(self.handle, _p(s), _p(p), n), "mpt_rrt_read_tree")
        return s, p

    def last_round(self, K: int):
        samples = np.zeros((K, self.dim))
        nn = np.zeros(K, np.int32)
        ends = np.zeros((K, self.dim))
        verdict = np.zeros(K, np.uint8)
        check(lib().mpt_rrt_last_round(self.handle, _p(samples), _p(nn), _p(ends), _p(verdict)), "mpt_rrt_last_round")
        return samples, nn, ends, verdict

    def info(self) -> dict:
        out = np.zeros(4, np.int64)
        check(lib().mpt_rrt_info(self.handle, _p(out)), "mpt_rrt_info")
        return {"dim": int(out[0]), "links": int(out[1]), "pmax": int(out[2]), "capacity": int(out[3])}

    def last_poses(self, K: int):
        inf = self.info()
        poses = np.zeros((K, inf["pmax"], inf["links"], 12))
        counts = np.zeros(K, np.int32)
        check(lib().mpt_rrt_last_poses(self.handle, _p(poses), _p(counts)), "mpt_rrt_last_poses")
        return poses, counts

    def last_nn(self) -> str:
        """NN structure the last round used: 'brute' | 'grid' | 'tree' ('' before any round)."""
        m = C.c_int32(-1)
        check(lib().mpt_rrt_last_nn(self.handle, C.byref(m)), "mpt_rrt_last_nn")
        return {1: "brute", 2: "grid", 3: "tree"}.get(m.value, "")

    def enable_timing(self, on: bool = True) -> None:
        check(lib().mpt_rrt_enable_timing(self.handle, 1 if on else 0), "mpt_rrt_enable_timing")

    def kernel_times(self) -> dict:
        ms = np.zeros(9, np.float32)
        check(lib().mpt_rrt_kernel_times(self.handle, _p(ms)), "mpt_rrt_kernel_times")
        names = ["sample", "nn_build", "nn_query", "steer", "collide_pairs", "collide_cands", "collide_narrow",
                 "collide_rest", "append"]
        t = dict(zip(names, ms.astype(float).tolist()))
        t["collide"] = t["collide_pairs"] + t["collide_cands"] + t["collide_narrow"] + t["collide_rest"]
        return t

    def kernel_times_sum(self) -> tuple:
        """(per-stage ms summed over the rounds recorded since the last call, rounds)."""
        ms = np.zeros(9, np.float64)
        n = np.zeros(1, np.int64)
        check(lib().mpt_rrt_kernel_times_sum(self.handle, _p(ms), _p(n)), "mpt_rrt_kernel_times_sum")
        names = ["sample", "nn_build", "nn_query", "steer", "collide_pairs", "collide_cands", "collide_narrow",
                 "collide_rest", "append"]
        t = dict(zip(names, ms.tolist()))
        t["collide"] = t["collide_pairs"] + t["collide_cands"] + t["collide_narrow"] + t["collide_rest"]
        return t, int(n[0])

    def collide_stats(self, enable: bool) -> dict:
        """Counters since the last call (then reset); enable keeps counting in later rounds."""
        out = np.zeros(16, np.uint64)
        check(lib().mpt_rrt_collide_stats(self.handle, 1 if enable else 0, _p(out)), "mpt_rrt_collide_stats")
        names = ["units", "clusters", "node_tests", "tri_tests", "pair_tests", "fused_reruns", "cluster_transforms",
                 "candidates", "nn_points", "nn_cells", "cluster_threads", "nn_steps"]
        return {k: int(v) for k, v in zip(names, out[:12])}

    def set_nn(self, mode: str = "auto", points_per_cell: float = 0.0) -> None:
        """NN structure of the rounds: 'auto' | 'brute' | 'grid' | 'tree' (identical results)."""
        check(lib().mpt_rrt_set_nn(self.handle, {"auto": 0, "brute": 1, "grid": 2, "tree": 3}[mode], points_per_cell),
              "mpt_rrt_set_nn")

    def close(self):
        if getattr(self, "handle", None):
            lib().mpt_rrt_destroy(self.handle)
            self.handle = None

    __del__ = close


# ---------------------------------------------------------------- host planner (C++)

def step_many(engines, K: int, streams, joint_stream=None) -> None:
    """One round of several independent engines (mpt_rrt_step_many): engine i on streams[i],
    the Morton-tree NN queries of all of them in one launch on joint_stream.  Results are
    those of engines[i].step(K, streams[i]) for every i."""
    n = len(engines)
    hs = (C.c_void_p * n)(*[e.handle.value if isinstance(e.handle, C.c_void_p) else e.handle for e in engines])
    ss = (C.c_void_p * n)(*[(_stream(s).value if s is not None else None) for s in streams])
    check(lib().mpt_rrt_step_many(hs, n, K, ss, _stream(joint_stream)), "mpt_rrt_step_many")


def joint_nn_ms() -> float:
    """hipEvent duration of this thread's last timed joint NN launch (step_many)."""
    ms = C.c_float()
    check(lib().mpt_rrt_joint_nn_ms(C.byref(ms)), "mpt_rrt_joint_nn_ms")
    return ms.value


def joint_times(joint_stream) -> dict:
    """The last timed step_many on joint_stream: {"build": ms of the joint tree build,
    "nn": ms of the joint NN launch} (hipEvents on that stream)."""
    ms = np.zeros(2, np.float32)
    check(lib().mpt_rrt_joint_times(_stream(joint_stream), _p(ms)), "mpt_rrt_joint_times")
    return {"build": float(ms[0]), "nn": float(ms[1])}


def joint_stage_times(joint_stream) -> dict:
    """The last step_many on joint_stream when it ran as a timed joint round: ms of each stage
    (one launch per stage for all engines, hipEvents on that stream)."""
    ms = np.zeros(6, np.float32)
    check(lib().mpt_rrt_joint_stage_times(_stream(joint_stream), _p(ms)), "mpt_rrt_joint_stage_times")
    return dict(zip(["sample", "nn_build", "nn_query", "steer", "collide", "append"], ms.astype(float).tolist()))


def joint_release(joint_stream) -> None:
    """Free the joint state step_many keeps for joint_stream (call before the stream goes)."""
    check(lib().mpt_rrt_joint_release(_stream(joint_stream)), "mpt_rrt_joint_release")

def joint_replay_nn(joint_stream, parts: int = 0) -> None:
    """Diagnostics: joint_stream's last joint NN launch again (same jobs; same results); parts:
    0 = each tree over all eight XCDs, P > 0 = each tree in P contiguous runs, one XCD each."""
    check(lib().mpt_rrt_joint_replay_nn(_stream(joint_stream), int(parts)), "mpt_rrt_joint_replay_nn")


def load_mesh(path: str, which: str = "all") -> np.ndarray:
    """AssimpMeshLoader replacement: 'all' submeshes (environment) or 'last' (agent)."""
    w = 1 if which == "last" else 0
    n = C.c_int64()
    ns = C.c_int32()
    check(lib().mpt_host_load_mesh(path.encode(), w, None, 0, C.byref(n), C.byref(ns)), "mpt_host_load_mesh",
          host=True)
    out = np.zeros((n.value, 9))
    check(lib().mpt_host_load_mesh(path.encode(), w, _p(out), n.value, C.byref(n), C.byref(ns)),
          "mpt_host_load_mesh", host=True)
    return out


def prm(path: str, states=None, batch: int = 1, max_queries: int = 50):
    """PRM (planners/prm/prm.hpp) via the C++ host planner on a .inst file.
    states given: the roadmap over these milestones only; otherwise PRM::query(start, goal)
    until solved.  Returns dict(edges [E][2] (target, source), costs [E], comp [n], solved, cost)."""
    st = None if states is None else np.ascontiguousarray(states, np.float64)
    n = 0 if st is None else st.shape[0]
    ne, nm = C.c_int64(), C.c_int64()
    solved, cost = C.c_int32(), C.c_double()
    check(lib().mpt_host_prm(path.encode(), _p(st), n, batch, max_queries, 0, None, None, C.byref(ne), 0, None,
                             C.byref(nm), C.byref(solved), C.byref(cost)), "mpt_host_prm", host=True)
    # the counts are known now; run again to fill arrays of that size (deterministic)
    cap, ccap = max(ne.value, 1), max(nm.value, 1)
    edges = np.zeros((cap, 2), np.int32)
    costs = np.zeros(cap)
    comp = np.zeros(ccap, np.int32)
    check(lib().mpt_host_prm(path.encode(), _p(st), n, batch, max_queries, cap, _p(edges), _p(costs), C.byref(ne),
                             ccap, _p(comp), C.byref(nm), C.byref(solved), C.byref(cost)), "mpt_host_prm", host=True)
    return {"edges": edges[: ne.value], "costs": costs[: ne.value], "comp": comp[: nm.value],
            "solved": bool(solved.value), "cost": cost.value}


def grid_discretization(path: str, sizes) -> tuple:
    """GridDiscretization of the .inst's workspace: (free [cells] bool, centers [cells][3])."""
    sz = _f64(sizes)
    n = C.c_int64()
    check(lib().mpt_host_grid_discretization(path.encode(), _p(sz), 0, None, None, C.byref(n)),
          "mpt_host_grid_discretization", host=True)
    free = np.zeros(n.value, np.uint8)
    centers = np.zeros((n.value, 3))
    check(lib().mpt_host_grid_discretization(path.encode(), _p(sz), n.value, _p(free), _p(centers), C.byref(n)),
          "mpt_host_grid_discretization", host=True)
    return free.astype(bool), centers


def prmlite(path: str, n_vertices: int, step: float = 0.1) -> tuple:
    """PRMLite over the .inst's workspace and agent: (vertices [V][12], edges [E][2] i < j)."""
    verts = np.zeros((n_vertices, 12))
    cap = max(n_vertices * (n_vertices - 1) // 2, 1)
    edges = np.zeros((cap, 2), np.int32)
    ne = C.c_int64()
    check(lib().mpt_host_prmlite(path.encode(), n_vertices, step, _p(verts), cap, _p(edges), C.byref(ne)),
          "mpt_host_prmlite", host=True)
    return verts, edges[: ne.value]


def rrt_inst(path: str, iterations_at_a_time: int, cap: int = 1 << 16):
    """Run the C++ host planner on a .inst file: returns (starts, ends, solved)."""
    n = C.c_int64()
    dim = C.c_int32()
    solved = C.c_int32()
    starts = np.zeros(cap * 16)
    ends = np.zeros(cap * 16)
    check(lib().mpt_host_rrt_inst(path.encode(), iterations_at_a_time, cap, starts.size, _p(starts), _p(ends), C.byref(n),
                                  C.byref(dim), C.byref(solved)), "mpt_host_rrt_inst", host=True)
    d = dim.value
    m = min(n.value, cap)
    return starts[: m * d].reshape(m, d), ends[: m * d].reshape(m, d), bool(solved.value)


def rrt_batched_inst(path: str, cap: int = 1 << 20) -> dict:
    """Planner <file.inst> in its batched throughput mode (the file sets `Batch Size`; keys in
    include/mpt_host.h mpt_host_rrt_batched): counters, wall time and tree 0."""
    out = np.zeros(4, np.int64)
    secs = C.c_double()
    n = C.c_int64()
    dim = C.c_int32()
    states = np.zeros(cap * 16)
    parents = np.zeros(cap, np.int32)
    check(lib().mpt_host_rrt_batched(path.encode(), _p(out), C.byref(secs), cap, states.size, _p(states), _p(parents),
                                     C.byref(n), C.byref(dim)), "mpt_host_rrt_batched", host=True)
    d, m = dim.value, min(n.value, cap)
    return {"rounds": int(out[0]), "checked": int(out[1]), "valid": int(out[2]), "solved_trees": int(out[3]),
            "seconds": secs.value, "tree0": (states[: m * d].reshape(m, d), parents[:m])}
