"""Workloads of BASELINE.json's configs, as data for the device path.

Parameters come from the reference's instance files (omnidirectional.inst, blimp.inst,
snake.inst) and agents (agents/blimp.hpp:152-160, agents/snake_trailers.hpp:170-179).
Meshes are the repo fixtures under tests/golden/meshes/ (generated from the reference's
mesh_models/ by tests/golden/make_meshes.py).  Substitutions, all documented in DESIGN.md:

* blimp env = model.dae (the single-room mesh; blimp.inst:15 names unit_box.dae);
* snake env = a synthetic corridor (snake.inst:16-17 puts its only box outside the workspace);
* PRM env = a tiled grid of model.dae rooms, ~200k triangles (apartment.dae is missing,
  .MISSING_LARGE_BLOBS:1).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MESH_DIR = os.environ.get("MPT_MESH_DIR", os.path.join(REPO, "tests", "golden", "meshes"))


def mesh_path(name: str) -> str:
    return os.path.join(MESH_DIR, name + ".obj")


def read_obj(path: str, which: str = "all") -> np.ndarray:
    """Minimal OBJ reader for the fixtures (float32 values widened to double); the product
    loader is the C++ one behind api.load_mesh, this one exists for host-only tooling."""
    verts = []
    groups: list[list[int]] = []
    cur: list[int] | None = None
    with open(path) as f:
        for line in f:
            if line.startswith("o ") or line.startswith("g "):
                cur = []
                groups.append(cur)
            elif line.startswith("v "):
                verts.append([float(np.float32(x)) for x in line.split()[1:4]])
            elif line.startswith("f "):
                idx = [int(x.split("/")[0]) - 1 for x in line.split()[1:]]
                if len(idx) == 3:
                    if cur is None:
                        cur = []
                        groups.append(cur)
                    cur.extend(idx)
    v = np.asarray(verts, np.float64)
    if which == "last":
        groups = [g for g in groups if g][-1:]
    idx = np.asarray([i for g in groups for i in g], np.int64)
    return v[idx].reshape(-1, 9)


def box_tris(center, half) -> np.ndarray:
    """12 triangles of an axis-aligned box."""
    c = np.asarray(center, np.float64)
    h = np.asarray(half, np.float64) * np.ones(3)
    corners = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float64) * h + c
    faces = [(0, 1, 3), (0, 3, 2), (4, 6, 7), (4, 7, 5), (0, 4, 5), (0, 5, 1),
             (2, 3, 7), (2, 7, 6), (0, 2, 6), (0, 6, 4), (1, 5, 7), (1, 7, 3)]
    return np.concatenate([corners[list(f)].reshape(1, 9) for f in faces])


def corridor_env(seed: int = 0, length: float = 100.0, half_width: float = 4.0, n_obstacles: int = 20) -> np.ndarray:
    """Synthetic corridor for the snake config: two walls of unit boxes along y at
    x = +-half_width, plus n_obstacles random unit boxes between them (seeded)."""
    rng = np.random.default_rng(seed)
    boxes = []
    ys = np.arange(-length / 2, length / 2 + 1e-9, 1.0)
    for x in (-half_width, half_width):
        for y in ys:
            boxes.append(box_tris((x, y, 0.0), 0.5))
    for _ in range(n_obstacles):
        boxes.append(box_tris((rng.uniform(-half_width + 1.5, half_width - 1.5), rng.uniform(-length / 2, length / 2),
                               0.0), 0.5))
    return np.concatenate(boxes)


def rooms_env(nx: int = 25, ny: int = 25) -> np.ndarray:
    """Synthetic multi-room environment: nx*ny copies of the model.dae room (316 tris),
    tiled on a 180 x 140 grid (the room spans 177.2 x 137.8 x 114.2)."""
    room = read_obj(mesh_path("env_model"))
    out = np.empty((nx * ny,) + room.shape)
    k = 0
    for i in range(nx):
        for j in range(ny):
            t = room.copy().reshape(-1, 3)
            t[:, 0] += 180.0 * i
            t[:, 1] += 140.0 * j
            out[k] = t.reshape(-1, 9)
            k += 1
    return out.reshape(-1, 9)


@dataclass
class Scenario:
    name: str
    kind: int                 # 0 omni, 1 blimp, 2 snake (include/mpt.h MPT_AGENT_*)
    prm: np.ndarray
    ranges: np.ndarray        # [d][2] = Agent::getStateVarRanges(Map3D::getBounds())
    steer_dt: float
    cc_dt: float
    env_tris: np.ndarray
    env_tf: np.ndarray
    agent_tris: np.ndarray
    start: np.ndarray
    goal: np.ndarray
    goal_thr: np.ndarray
    links: int = 1
    notes: dict = field(default_factory=dict)

    @property
    def dim(self) -> int:
        return self.ranges.shape[0]


IDENTITY_TF = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], np.float64)


def omni_scenario() -> Scenario:
    """omnidirectional.inst: unit box agent vs unit box env at the origin, bounds [-10,10]^3."""
    bounds = np.array([[-10, 10], [-10, 10], [-10, 10]], np.float64)
    return Scenario("omnidirectional", 0, np.zeros(7), bounds, 0.1, 0.1,
                    read_obj(mesh_path("env_unit_box")), IDENTITY_TF.copy(),
                    read_obj(mesh_path("agent_unit_box"), "last"),
                    np.array([-5.0, -5.0, 0.0]), np.array([5.0, 5.0, 0.0]), np.array([1.0, 1.0, 1.0]))


BLIMP_PRM = np.array([10.0, -1.0, 5.0, -0.785398, 0.785398, -5.0, 5.0])  # blimp.inst:7-13


def blimp_ranges(bounds=((-100, 100), (-100, 100), (-100, 100)), prm=BLIMP_PRM) -> np.ndarray:
    b = [list(x) for x in bounds]  # Blimp::getStateVarRanges (agents/blimp.hpp:152-160)
    return np.array(b + [[0.0, 2 * math.pi], [prm[1], prm[2]], [prm[3], prm[4]], [prm[5], prm[6]]], np.float64)


def blimp_scenario(agent_submeshes: str = "all") -> Scenario:
    """blimp.inst with the single-room env (model.dae).  agent_submeshes='all' uses the
    whole blimp.3ds soup (1355 tris, the throughput workload); 'last' is the reference
    SimpleAgentMeshHandler behaviour (last submesh, 32 tris)."""
    return Scenario("blimp", 1, BLIMP_PRM.copy(), blimp_ranges(), 0.1, 0.1,
                    read_obj(mesh_path("env_model")), IDENTITY_TF.copy(),
                    read_obj(mesh_path("agent_blimp"), agent_submeshes),
                    np.array([0, 0, 0, 1, 0, 0, 0], np.float64), np.array([5, 5, 0, 1, 0, 0, 0], np.float64),
                    np.array([1.0, 1.0, 1.0]), notes={"agent_submeshes": agent_submeshes})


def blimp_room_scenario(agent_submeshes: str = "all") -> Scenario:
    """The collision-heavy config-2 variant (BASELINE config 2 "with poses drawn
    from the tree"): blimp.inst's agent and dynamics in model.dae, with the sampling box's
    x, y, z ranges = the room's bounding box (0-177.2 x 0-137.8 x 0-114.2) instead of
    blimp.inst:17's [-100, 100]^3, so every pose lies in the room and reaches the narrow phase."""
    sc = blimp_scenario(agent_submeshes)
    v = sc.env_tris.reshape(-1, 3)
    sc.ranges = blimp_ranges(tuple(zip(v.min(0).tolist(), v.max(0).tolist())))
    sc.name = "blimp-room"
    return sc


SNAKE_PRM = np.array([10, 1.0, 0.25, -1.0, 5.0, -0.785398, 0.785398])  # snake.inst:7-15


def snake_scenario(env: str = "corridor") -> Scenario:
    T = int(SNAKE_PRM[0])
    ranges = np.array([[-50, 50], [-50, 50], [SNAKE_PRM[3], SNAKE_PRM[4]], [SNAKE_PRM[5], SNAKE_PRM[6]]]
                      + [[0.0, 2 * math.pi]] * (T + 1), np.float64)
    if env == "corridor":
        env_tris, tf = corridor_env(0), IDENTITY_TF.copy()
    else:  # the reference's snake.inst: unit box at (-100, 0, 0)
        env_tris = read_obj(mesh_path("env_unit_box"))
        tf = IDENTITY_TF.copy()
        tf[9] = -100.0
    start = np.zeros(5 + T)
    goal = np.zeros(5 + T)
    goal[1] = 20.0
    return Scenario("snake", 2, SNAKE_PRM.copy(), ranges, 0.25, 1.0, env_tris, tf,
                    read_obj(mesh_path("agent_unit_box"), "last"), start, goal, np.array([1.0, 1.0]), links=T + 1)
