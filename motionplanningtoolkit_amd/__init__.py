"""motionplanningtoolkit_amd -- the RRT/PRM inner loop of csbence/motionplanningtoolkit
(batched FCL-semantics mesh collision + FLANN-semantics nearest neighbours) as HIP
kernels for MI355X (gfx950) behind a C ABI (include/mpt.h), with the reference's
Agent / Sampler / TreeInterface / `.inst` surface kept in C++ (csrc/host/).

See DESIGN.md for the path, the data layout and the kernels.
"""
from ._native import LIB_PATH, MptError, build, lib  # noqa: F401
from .api import (  # noqa: F401
    AGENT_BLIMP,
    AGENT_OMNI,
    AGENT_SNAKE,
    AgentMesh,
    Environment,
    NearestNeighbors,
    RRTEngine,
    collide_batch,
    collide_batch_device,
    distance_batch,
    distance_batch_device,
    init,
    joint_nn_ms,
    joint_release,
    joint_stage_times,
    prm_stats,
    joint_times,
    last_collide_stats,
    load_mesh,
    prm,
    prm_connect,
    prmlite_edges,
    prmlite,
    grid_discretization,
    rrt_batched_inst,
    rrt_inst,
    prm_deferred_edges,
    joint_replay_nn,
    set_collide_mode,
    set_sweep_queue_cap,
    set_collide_stats,
    step_many,
    synchronize,
    transform_from_location,
)

__all__ = [
    "AGENT_OMNI", "AGENT_BLIMP", "AGENT_SNAKE", "AgentMesh", "Environment", "NearestNeighbors", "RRTEngine",
    "collide_batch", "collide_batch_device", "distance_batch", "distance_batch_device", "init", "joint_nn_ms", "joint_release", "joint_replay_nn", "joint_stage_times", "prm_stats", "prm_deferred_edges", "joint_times", "last_collide_stats", "load_mesh", "prm", "prm_connect", "prmlite_edges", "prmlite", "grid_discretization", "rrt_inst", "rrt_batched_inst",
    "set_collide_mode", "set_sweep_queue_cap", "set_collide_stats", "step_many", "synchronize", "transform_from_location", "build", "lib", "LIB_PATH", "MptError",
]
