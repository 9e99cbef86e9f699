"""GPU parity for config 4 (PRM with radius neighbours, mpt_prm_connect): point-tree radius
search, edge poses and batched collision against the oracle's restatement (orc_prm_radius).
Bar: identical edge lists, verdicts and components."""
import numpy as np
import pytest

from motionplanningtoolkit_amd import scenes

pytestmark = pytest.mark.gpu

I12 = np.r_[np.eye(3).ravel(), 0.0, 0.0, 0.0]


def compare(mpt, oracle, env_tris, agent_tris, kind, states, r2, cc_dt, env_tf=I12):
    env, ag = mpt.Environment(env_tris, env_tf), mpt.AgentMesh(agent_tris)
    got = mpt.prm_connect(env, ag, kind, states, r2, cc_dt)
    edges, verdict, comp = oracle.prm_radius(oracle.BVH(env_tris), env_tf, agent_tris, states, r2, cc_dt)
    assert got["edges"].shape == edges.shape, (got["edges"].shape, edges.shape)
    assert np.array_equal(got["edges"], edges)
    assert np.array_equal(got["verdict"], verdict), np.nonzero(got["verdict"] != verdict)
    assert np.array_equal(got["comp"], comp)
    return got


def test_omni_unit_box(mpt_gpu, oracle):
    box = scenes.read_obj(scenes.mesh_path("agent_unit_box"), "last")
    st = np.random.default_rng(1).uniform(-6, 6, (1500, 3))
    got = compare(mpt_gpu, oracle, box, box, 0, st, 2.5 ** 2, 0.1)
    assert 0 < got["verdict"].sum() < len(got["verdict"])


def test_omni_corridor(mpt_gpu, oracle):
    box = scenes.read_obj(scenes.mesh_path("agent_unit_box"), "last")
    env = scenes.read_obj(scenes.mesh_path("env_corridor"))
    rng = np.random.default_rng(2)
    st = np.stack([rng.uniform(-6, 6, 2000), rng.uniform(-52, 52, 2000), rng.uniform(-1, 1, 2000)], 1)
    got = compare(mpt_gpu, oracle, env, box, 0, st, 4.0 ** 2, 0.1)
    assert len(np.unique(got["comp"])) > 1


@pytest.mark.parametrize("agent_mode", ["last", "all"])
@pytest.mark.parametrize("mode", ["split", "fused"])
def test_blimp_room(mpt_gpu, oracle, agent_mode, mode):
    """split: the sweep with each edge's poses generated in the kernel (prm_edges.h, no pose
    array); fused: the pose array and the per-pose walk -- the same verdicts."""
    sc = scenes.blimp_scenario(agent_mode)
    rng = np.random.default_rng(3)
    n = 1200
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, 7))
    st[:, :3] = rng.uniform([-10, -10, -10], [190, 150, 125], size=(n, 3))
    mpt_gpu.set_collide_mode(mode)
    try:
        got = compare(mpt_gpu, oracle, sc.env_tris, sc.agent_tris, 1, st, 14.0 ** 2, sc.cc_dt)
    finally:
        mpt_gpu.set_collide_mode("split")
    assert 0 < got["verdict"].sum() < len(got["verdict"])


def test_agent_of_many_clusters(mpt_gpu, oracle):
    """An agent of more than 64 clusters (four copies of the blimp, 5420 triangles, 85
    clusters): the sweep's one-wave-an-(edge, cluster) form with in-kernel poses."""
    sc = scenes.blimp_scenario("all")
    ag = np.concatenate([sc.agent_tris + np.array([dx, 0, 0] * 3) for dx in (0.0, 3.0, 6.0, 9.0)])
    assert len(ag) > 64 * 64  # clusters hold at most 64 triangles (mpt_agent_create)
    rng = np.random.default_rng(8)
    n = 300
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, 7))
    st[:, :3] = rng.uniform([-10, -10, -10], [190, 150, 125], size=(n, 3))
    got = compare(mpt_gpu, oracle, sc.env_tris, ag, 1, st, 20.0 ** 2, sc.cc_dt)
    assert 0 < got["verdict"].sum() < len(got["verdict"])


def test_multi_room_env(mpt_gpu, oracle):
    """A deeper env tree (4 x 3 rooms, 3792 triangles)."""
    sc = scenes.blimp_scenario("last")
    env = scenes.rooms_env(4, 3)
    rng = np.random.default_rng(6)
    n = 1500
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, 7))
    st[:, :3] = rng.uniform([-10, -10, -10], [730, 430, 125], size=(n, 3))
    compare(mpt_gpu, oracle, env, sc.agent_tris, 1, st, 30.0 ** 2, sc.cc_dt)


def test_empty_and_isolated(mpt_gpu, oracle):
    box = scenes.read_obj(scenes.mesh_path("agent_unit_box"), "last")
    env, ag = mpt_gpu.Environment(box, I12), mpt_gpu.AgentMesh(box)
    one = mpt_gpu.prm_connect(env, ag, 0, np.array([[5.0, 5.0, 5.0]]), 1.0, 0.1)
    assert len(one["edges"]) == 0 and list(one["comp"]) == [0]
    far = mpt_gpu.prm_connect(env, ag, 0, np.array([[5.0, 5, 5], [9, 9, 9], [5, 5, 5.5]]), 1.0, 0.1)
    assert far["edges"].tolist() == [[2, 0]] and far["comp"].tolist() == [0, 1, 0]


def _rotation(axis, angle):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * K @ K


@pytest.mark.parametrize("offset", [(2500.0, -1800.0, 900.0), (-40000.0, 65000.0, 12000.0)])
def test_rotated_env_large_coordinates(mpt_gpu, oracle, offset):
    """The sweep's per-(triangle, env triangle) pose interval (prm_edges.h near_range) is a float
    bound on the env-relative translation R_env^T (s + i step dx - T_env): under a rotated env
    transform its terms cancel, so the interval's slack must follow the terms' magnitudes (|d|,
    step it |dx|), not the sums'.  A tilted rotation and large world coordinates: the milestones
    are the rooms' local points carried into the world by the env transform, so the edges cross
    the walls as in the identity case, with every rotated sum a cancellation of large terms."""
    sc = scenes.blimp_scenario("last")
    env = scenes.rooms_env(4, 3)
    R = _rotation([0.3, -0.5, 0.81], 0.73)
    tf = np.r_[R.ravel(), np.asarray(offset)]
    rng = np.random.default_rng(12)
    n = 1500
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, 7))
    local = rng.uniform([-10, -10, -10], [730, 430, 125], size=(n, 3))
    st[:, :3] = local @ R.T + np.asarray(offset)  # world = R local + T (the env's own transform)
    got = compare(mpt_gpu, oracle, env, sc.agent_tris, 1, st, 30.0 ** 2, sc.cc_dt, env_tf=tf)
    assert 0.02 < got["verdict"].mean() < 0.98


def test_full_queue_path(mpt_gpu, oracle):
    """The sweep's candidate queue capped at a few entries (mpt_set_sweep_queue_cap): edges find
    it full and go to the per-edge pass (the fused list, k_sweep_prm<1>) -- the path a roadmap
    reaches only past ~4 M queued candidates -- with verdicts identical to the oracle's and to
    the uncapped call's."""
    sc = scenes.blimp_scenario("all")
    rng = np.random.default_rng(3)
    n = 1200
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, 7))
    st[:, :3] = rng.uniform([-10, -10, -10], [190, 150, 125], size=(n, 3))
    env, ag = mpt_gpu.Environment(sc.env_tris, I12), mpt_gpu.AgentMesh(sc.agent_tris)
    free = mpt_gpu.prm_connect(env, ag, 1, st, 14.0 ** 2, sc.cc_dt)
    mpt_gpu.set_sweep_queue_cap(16)
    try:
        mpt_gpu.prm_stats(True)
        got = compare(mpt_gpu, oracle, sc.env_tris, sc.agent_tris, 1, st, 14.0 ** 2, sc.cc_dt)
        work = mpt_gpu.prm_stats(False)
        deferred = mpt_gpu.prm_deferred_edges()
    finally:
        mpt_gpu.set_sweep_queue_cap(0)
        mpt_gpu.prm_stats(False)
    assert np.array_equal(got["verdict"], free["verdict"])
    assert work["deferred_edges"] == len(deferred) > 10, (work, len(deferred))
    assert len(np.unique(deferred)) == len(deferred) and deferred.max() < len(got["edges"])
    with pytest.raises(mpt_gpu.MptError):
        mpt_gpu.set_sweep_queue_cap(-1)
