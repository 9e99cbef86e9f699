"""ctypes binding of libmpt.so (include/mpt.h, include/mpt_host.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
motionplanningtoolkit_amd/csrc``) into ``motionplanningtoolkit_amd/_lib/libmpt.so``.
There is no fallback: if the library is missing or was built for another target,
``lib()`` raises, and every compute entry point returns an error status on a machine
without a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libmpt.so")
CSRC = os.path.join(_HERE, "csrc")

_lib = None

P = C.c_void_p
I32 = C.c_int32
I64 = C.c_int64
U64 = C.c_uint64
D = C.c_double

# name -> (restype, argtypes); every symbol declared in include/mpt.h and include/mpt_host.h
SIGNATURES = {
    "mpt_init": (I32, [I32]),
    "mpt_last_error": (C.c_char_p, []),
    "mpt_version": (I32, []),
    "mpt_device_synchronize": (I32, []),
    "mpt_env_create": (I32, [P, I64, P, P]),
    "mpt_env_destroy": (I32, [P]),
    "mpt_env_info": (I32, [P, P]),
    "mpt_agent_create": (I32, [P, I64, P]),
    "mpt_agent_destroy": (I32, [P]),
    "mpt_transform_from_location": (I32, [P, P]),
    "mpt_collide_batch": (I32, [P, P, I32, P, P, I64, P, P]),
    "mpt_collide_batch_device": (I32, [P, P, I32, P, P, I64, I64, P, P]),
    "mpt_collide_batch_ex": (I32, [P, P, I32, P, P, I64, I32, P, P]),
    "mpt_set_stats": (I32, [I32]),
    "mpt_set_collide_mode": (I32, [I32]),
    "mpt_distance_batch": (I32, [P, P, I32, P, P, I64, P, P]),
    "mpt_prm_connect": (I32, [P, P, I32, P, I64, I32, D, D, I64, P, P, P, P, P]),
    "mpt_prmlite_edges": (I32, [P, P, P, I64, D, P, P]),
    "mpt_distance_batch_device": (I32, [P, P, I32, P, P, I64, I64, P, P]),
    "mpt_last_collide_stats": (I32, [P]),
    "mpt_nn_create": (I32, [I32, I64, P]),
    "mpt_nn_destroy": (I32, [P]),
    "mpt_nn_append": (I32, [P, P, I64, P]),
    "mpt_nn_append_device": (I32, [P, P, I64, P]),
    "mpt_nn_remove": (I32, [P, I32]),
    "mpt_nn_size": (I32, [P, P]),
    "mpt_nn_points_device": (I32, [P, P]),
    "mpt_nn_set_index": (I32, [P, I32]),
    "mpt_nn_knn": (I32, [P, P, I64, I32, P, P, P]),
    "mpt_nn_knn_device": (I32, [P, P, I64, I32, P, P, P]),
    "mpt_nn_radius": (I32, [P, P, I64, D, I32, P, P, P, I64, P]),
    "mpt_rrt_create": (I32, [P, P, I32, P, P, I32, D, D, I64, U64, P]),
    "mpt_rrt_destroy": (I32, [P]),
    "mpt_rrt_add_nodes": (I32, [P, P, P, I64]),
    "mpt_rrt_set_size": (I32, [P, I64, P]),
    "mpt_rrt_step": (I32, [P, I32, P]),
    "mpt_rrt_step_many": (I32, [P, I32, I32, P, P]),
    "mpt_rrt_joint_nn_ms": (I32, [P]),
    "mpt_rrt_joint_times": (I32, [P, P]),
    "mpt_rrt_joint_release": (I32, [P]),
    "mpt_rrt_joint_replay_nn": (I32, [P, I32]),
    "mpt_rrt_joint_stage_times": (I32, [P, P]),
    "mpt_prm_stats": (I32, [I32, P, I32]),
    "mpt_set_sweep_queue_cap": (I32, [I64]),
    "mpt_prm_deferred_edges": (I32, [P, I64, P]),
    "mpt_rrt_counters": (I32, [P, P]),
    "mpt_rrt_read_tree": (I32, [P, P, P, I64]),
    "mpt_rrt_last_round": (I32, [P, P, P, P, P]),
    "mpt_rrt_last_poses": (I32, [P, P, P]),
    "mpt_rrt_info": (I32, [P, P]),
    "mpt_rrt_last_nn": (I32, [P, P]),
    "mpt_rrt_enable_timing": (I32, [P, I32]),
    "mpt_rrt_set_nn": (I32, [P, I32, D]),
    "mpt_rrt_collide_stats": (I32, [P, I32, P]),
    "mpt_rrt_kernel_times": (I32, [P, P]),
    "mpt_rrt_kernel_times_sum": (I32, [P, P, P]),
    "mpt_host_last_error": (C.c_char_p, []),
    "mpt_host_load_mesh": (I32, [C.c_char_p, I32, P, I64, P, P]),
    "mpt_host_rrt_inst": (I32, [C.c_char_p, I32, I64, I64, P, P, P, P, P]),
    "mpt_host_rrt_batched": (I32, [C.c_char_p, P, P, I64, I64, P, P, P, P]),
    "mpt_host_prm": (I32, [C.c_char_p, P, I64, I32, I32, I64, P, P, P, I64, P, P, P, P]),
    "mpt_host_grid_discretization": (I32, [C.c_char_p, P, I64, P, P, P]),
    "mpt_host_prmlite": (I32, [C.c_char_p, I32, D, P, I64, P, P]),
}


class MptError(RuntimeError):
    def __init__(self, status: int, where: str, message: str):
        super().__init__(f"{where} failed with status {status}: {message}")
        self.status = status


def build(jobs: int = 8) -> str:
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True)
    return LIB_PATH


def lib():
    """Load libmpt.so (raises if it has not been built: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with __graft_entry__.build() or make -C {CSRC}")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int, where: str, host: bool = False) -> None:
    if status != 0:
        L = lib()
        msg = (L.mpt_host_last_error() if host else L.mpt_last_error()) or b""
        raise MptError(status, where, msg.decode(errors="replace"))
