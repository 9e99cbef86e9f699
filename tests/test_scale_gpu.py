"""GPU parity at the BASELINE configurations' full sizes.

* Config 2: one engine round of the benchmark's exact shape -- 100 000-node blimp tree,
  K = 65 536 extensions, blimp (1355 tris) vs the room (model.dae) -- NN ids of every query
  against the oracle's exact kd-tree, collision verdicts of every extension against the
  oracle's AABB-tree collider (on the device's own poses), and the ordered append.
* Config 3: the same at the snake leg's shape (100 000-node 15-dim tree, 11 links, corridor).
* Config 2, collision-heavy variant (`bench.py --workload blimp-room`): tree and samples
  inside the room, so every unit reaches the narrow phase; all 65 536 verdicts checked.
* Config 4: the 25 x 25-room environment (197 500 triangles, a four-level env tree that does
  not fit the k_pairs LDS stage) with 100 000 milestones over the whole multi-room extent:
  the roadmap of a milestone prefix against orc_prm_radius (edges, verdicts), the full edge
  set against scipy's cKDTree (pairs within 1e-9 relative of the radius are excluded: FLANN's
  summation order and cKDTree's differ there), the components against a host union-find, and
  mpt_collide_batch against orc_collide_batch_bvh on 4096 poses spread over the rooms.
Bars as everywhere: ids, verdicts, edge lists and components bit-exact.
"""
import math
import os

import numpy as np
import pytest

from motionplanningtoolkit_amd import scenes

pytestmark = pytest.mark.gpu

THREADS = min(16, len(os.sched_getaffinity(0)))
I12 = np.r_[np.eye(3).ravel(), 0.0, 0.0, 0.0]


def _engine_round_check(mpt, oracle, sc, tree, K, seed, n_sample=4096, nn_mode=None):
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    ag = mpt.AgentMesh(sc.agent_tris)
    n0 = len(tree)
    eng = mpt.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, n0 + K, seed)
    eng.add_nodes(tree)
    eng.step(K)
    if nn_mode:
        assert eng.last_nn() == nn_mode
    samples, nn, ends, verdict = eng.last_round(K)
    poses, pcount = eng.last_poses(K)
    # samples: the counter-based generator (spot check, pure +,-,* arithmetic)
    for k in (0, 1, K // 2, K - 1):
        exp = [oracle.engine_uniform(seed, k * 64 + j, lo, hi) for j, (lo, hi) in enumerate(sc.ranges)]
        assert np.array_equal(samples[k], np.array(exp))
    # NN ids of every query (exact kd-tree with FLANN's distance order, ties to the lowest id)
    ref_ids, _ = oracle.KDTree(tree).knn(samples, 1, nthreads=THREADS)
    assert np.array_equal(nn, ref_ids[:, 0])
    # verdicts of a sample of extensions, on the device's own poses
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(K, size=min(n_sample, K), replace=False))
    L = sc.links
    flat = np.concatenate([poses[k, :pcount[k]] for k in idx]).reshape(-1, L, 12)
    off = np.r_[0, np.cumsum(pcount[idx])]
    ref_v = oracle.collide_batch_bvh(oracle.BVH(sc.env_tris), sc.env_tf, [sc.agent_tris] * L, flat, off,
                                     nthreads=THREADS)
    assert np.array_equal(verdict[idx], ref_v)
    # ordered append of the collision-free extensions
    valid = np.nonzero(verdict == 0)[0]
    c = eng.counters()
    assert c["nodes"] == n0 + len(valid)
    t2, par = eng.read_tree(n0 + len(valid))
    assert np.array_equal(t2[:n0], tree)
    assert np.array_equal(t2[n0:], ends[valid]) and np.array_equal(par[n0:], nn[valid])
    return verdict


def test_config2_full_round(mpt_gpu, oracle):
    sc = scenes.blimp_scenario("all")
    seed = 1000  # bench.py's rank-0 seed
    tree = np.random.default_rng(seed).uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(100_000, sc.dim))
    v = _engine_round_check(mpt_gpu, oracle, sc, tree, 65_536, seed, n_sample=65_536, nn_mode="grid")
    assert 0 < v.sum() < len(v)


def test_config3_full_round(mpt_gpu, oracle):
    """Config 3 at the bench's snake shape (`bench.py --workload snake`): snake_trailers (11
    unit-box links, d = 15) in the synthetic corridor, a 100 000-node tree over the snake's
    state ranges, K = 65 536 -- the grid NN over x, y with the head screen
    (k_grid_nn1_runs_sorted<15, ...>).  Every NN id against the oracle's exact kd-tree, the
    verdicts of all 65 536 extensions on the device's poses (all 11 links) against the oracle's
    AABB-tree collider, and the ordered append (snake_trailers.hpp:170-183, 246-268)."""
    sc = scenes.snake_scenario("corridor")
    seed = 1000
    tree = np.random.default_rng(seed).uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(100_000, sc.dim))
    v = _engine_round_check(mpt_gpu, oracle, sc, tree, 65_536, seed, n_sample=65_536, nn_mode="grid")
    assert 0 < v.sum() < len(v)


def test_config2_room_full_round(mpt_gpu, oracle):
    """The collision-heavy variant: every pose inside the room's box; the verdicts of all
    65 536 extensions against the oracle (every unit reaches the narrow phase here)."""
    sc = scenes.blimp_room_scenario()
    seed = 1000
    tree = np.random.default_rng(seed).uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(100_000, sc.dim))
    v = _engine_round_check(mpt_gpu, oracle, sc, tree, 65_536, seed, n_sample=65_536)
    assert v.mean() > 0.05  # a real collision workload


def rooms_prm_inputs(n=100_000, rooms=25, degree=10.0, seed=0):
    """Config 4 milestones over the whole multi-room extent (scripts/bench_prm.py --bounds rooms)."""
    sc = scenes.blimp_scenario("all")
    env_t = scenes.rooms_env(rooms, rooms)
    lo = env_t.reshape(-1, 3).min(0)
    hi = env_t.reshape(-1, 3).max(0)
    rng = np.random.default_rng(seed)
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n, sc.dim))
    st[:, :3] = rng.uniform(lo, hi, size=(n, 3))
    vol = float(np.prod(hi - lo))
    r = (degree * vol / (n * 4.0 / 3.0 * math.pi)) ** (1.0 / 3.0)
    return sc, env_t, st, r * r


def _components(n, edges, verdict):
    parent = np.arange(n)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a

    for (i, j), v in zip(edges, verdict):
        if v == 0:
            a, b = find(int(i)), find(int(j))
            if a != b:
                parent[max(a, b)] = min(a, b)
    return np.array([find(i) for i in range(n)], np.int32)


def test_config4_rooms_at_size(mpt_gpu, oracle):
    from scipy.spatial import cKDTree

    sc, env_t, st, r2 = rooms_prm_inputs()
    assert env_t.shape[0] == 197_500
    env, ag = mpt_gpu.Environment(env_t, I12), mpt_gpu.AgentMesh(sc.agent_tris)
    got = mpt_gpu.prm_connect(env, ag, 1, st, r2, sc.cc_dt)
    edges, verdict = got["edges"], got["verdict"]
    n = len(st)
    assert len(edges) > 300_000 and 0 < verdict.sum() < len(verdict)
    # (1) the whole edge set: pairs (i, j), j < i, of squared key distance < r2
    keys = st[:, :3]
    pairs = cKDTree(keys).query_pairs(math.sqrt(r2) * (1 + 1e-9), output_type="ndarray")
    d2 = ((keys[pairs[:, 0]] - keys[pairs[:, 1]]) ** 2).sum(1)
    clear = np.abs(d2 - r2) > 1e-9 * r2
    exp = set(map(tuple, np.sort(pairs[clear & (d2 < r2)], axis=1)[:, ::-1].tolist()))
    amb = set(map(tuple, np.sort(pairs[~clear], axis=1)[:, ::-1].tolist()))
    got_set = set(map(tuple, edges.tolist()))
    assert exp <= got_set and got_set - exp <= amb
    # edges sorted by i, then j (the C ABI's order)
    key = edges[:, 0].astype(np.int64) * n + edges[:, 1]
    assert np.all(np.diff(key) > 0)
    # (2) a milestone prefix against the oracle's restatement: edges and verdicts identical
    #     (the oracle checks ~260 poses of the 1355-triangle blimp per edge: ~40 ms per edge)
    k = 4_000
    e_ref, v_ref, _ = oracle.prm_radius(oracle.BVH(env_t), I12, sc.agent_tris, st[:k], r2, sc.cc_dt,
                                        nthreads=THREADS)
    pre = edges[:, 0] < k
    assert len(e_ref) > 400
    assert np.array_equal(edges[pre], e_ref)
    assert np.array_equal(verdict[pre], v_ref)
    # (3) 10 000 edges drawn from the whole roadmap, up to half of them among the edges the
    #     sweep's candidate pass capped or a full queue deferred (mpt_prm_deferred_edges: the
    #     k_sweep_prm edges, the most candidates), the rest uniform: the oracle's verdict of each,
    #     from orc_prm_radius calls over their endpoints in index order, 1 000 drawn edges a call
    #     (an edge's poses depend on its two milestones only; edges among a call's endpoints that
    #     were not drawn are ignored)
    mpt_gpu.prm_stats(True)
    try:
        again = mpt_gpu.prm_connect(env, ag, 1, st, r2, sc.cc_dt)
        deferred = mpt_gpu.prm_deferred_edges()
    finally:
        mpt_gpu.prm_stats(False)
    assert np.array_equal(again["verdict"], verdict)
    assert len(deferred) > 1000, len(deferred)
    rng = np.random.default_rng(7)
    hard = rng.choice(deferred, size=min(5000, len(deferred)), replace=False)
    rest = np.setdiff1d(np.arange(len(edges)), hard)
    pick = np.concatenate([hard, rng.choice(rest, size=10_000 - len(hard), replace=False)])
    got_v = np.empty(len(pick), np.uint8)
    ref_v = np.empty(len(pick), np.uint8)
    bvh = oracle.BVH(env_t)
    for c0 in range(0, len(pick), 1000):
        sub = pick[c0:c0 + 1000]
        ends = np.unique(edges[sub].ravel())
        pos = np.full(n, -1, np.int64)
        pos[ends] = np.arange(len(ends))
        e_sub, v_sub, _ = oracle.prm_radius(bvh, I12, sc.agent_tris, st[ends], r2, sc.cc_dt, nthreads=THREADS)
        ref = {(int(a), int(b)): int(v) for (a, b), v in zip(e_sub.tolist(), v_sub.tolist())}
        drawn = [(int(pos[i]), int(pos[j])) for i, j in edges[sub].tolist()]
        assert all(d in ref for d in drawn)
        ref_v[c0:c0 + len(sub)] = [ref[d] for d in drawn]
        got_v[c0:c0 + len(sub)] = verdict[sub]
    assert np.array_equal(got_v, ref_v)
    assert 0 < ref_v[:len(hard)].sum() < len(hard) and 0 < ref_v[len(hard):].sum() < len(pick) - len(hard)
    # (4) components over the free edges
    assert np.array_equal(got["comp"], _components(n, edges, verdict))


def test_config4_rooms_collide_batch(mpt_gpu, oracle):
    """mpt_collide_batch in the 197 500-triangle env: 4096 single-pose edges (random yaw)
    spread over the rooms, half of them near a wall."""
    sc, env_t, _, _ = rooms_prm_inputs(n=10)
    env, ag = mpt_gpu.Environment(env_t, I12), mpt_gpu.AgentMesh(sc.agent_tris)
    rng = np.random.default_rng(11)
    P = 4096
    lo, hi = env_t.reshape(-1, 3).min(0), env_t.reshape(-1, 3).max(0)
    xyz = rng.uniform(lo, hi, size=(P, 3))
    # half of the poses within a few units of a random env vertex
    v = env_t.reshape(-1, 3)[rng.integers(0, env_t.shape[0] * 3, size=P // 2)]
    xyz[: P // 2] = v + rng.uniform(-6, 6, size=(P // 2, 3))
    th = rng.uniform(0, 2 * math.pi, P)
    poses = np.zeros((P, 12))
    poses[:, 0], poses[:, 1], poses[:, 3], poses[:, 4], poses[:, 8] = np.cos(th), np.sin(th), -np.sin(th), np.cos(th), 1
    poses[:, 9:] = xyz
    off = np.arange(P + 1, dtype=np.int64)
    for mode in ("split", "fused"):
        mpt_gpu.set_collide_mode(mode)
        try:
            got = mpt_gpu.collide_batch(env, [ag], poses.reshape(P, 1, 12), off)
        finally:
            mpt_gpu.set_collide_mode("split")
        ref = oracle.collide_batch_bvh(oracle.BVH(env_t), I12, [sc.agent_tris], poses.reshape(P, 1, 12), off,
                                       nthreads=THREADS)
        assert np.array_equal(got, ref), mode
        assert 0.05 < got.mean() < 0.95


def test_config5_shard_shape(mpt_gpu, oracle):
    """Config 5 at one GPU's shard (BASELINE config 5: 256 seeds, 32 per GPU): 32 blimp seeds
    from wall starts (bench.py --seed-start walls), 4096 extensions per seed per round, 30
    rounds through mpt_rrt_step_many (one joint Morton-tree build + NN launch per round; the
    trees reach ~110k nodes and the index is updated incrementally), exactly as bench.py
    --seeds 32 runs them.  Three seeds' trees are then grown by the oracle's engine rounds
    (orc_engine_step: kd-tree NN, correctly rounded steering trig, AABB-tree + FCL SAT; the
    reference's RRT::query loop, planners/rrt.hpp:42-94, batched) from the same starts and
    must equal the device's node for node, states and parents bitwise."""
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    sc = scenes.blimp_scenario("all")
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, base = 4096, 30, 1000
    seeds = [base + i for i in range(32)]
    starts = {s: bench.seed_start(s, env, ag, mpt_gpu, "walls") for s in seeds}
    engs = []
    for s in seeds:
        e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
        e.add_nodes(starts[s])
        e.set_nn("auto")
        engs.append(e)
    streams = [torch.cuda.Stream() for _ in range(8)]
    joint = torch.cuda.Stream()
    for _ in range(rounds):
        mpt_gpu.step_many(engs, K, [streams[j % 8] for j in range(len(engs))], joint)
    torch.cuda.synchronize()
    got = {}
    for s, e in zip(seeds, engs):
        assert e.last_nn() == "tree"
        got[s] = e.read_tree(e.counters()["nodes"])
        e.close()
    mpt_gpu.joint_release(joint)
    sizes = [len(got[s][0]) for s in seeds]
    assert min(sizes) > 60_000, sizes
    # the driver line's seeds=32 digest (same seeds, rounds and starts)
    import hashlib

    from motionplanningtoolkit_amd import multiseed

    assert rounds == bench.C5_WARMUP + bench.C5_STEPS
    dg = hashlib.sha256("".join(multiseed.tree_digest(*got[s]) for s in seeds).encode()).hexdigest()
    assert dg == _c5_golden()["seeds32"]
    bvh = oracle.BVH(sc.env_tris)
    for s in (seeds[0], seeds[13], seeds[31]):
        ref = np.zeros((1 + rounds * K, sc.dim))
        ref[0] = starts[s][0]
        par = np.zeros(1 + rounds * K, np.int32)
        n = 1
        for r in range(rounds):
            n, _, _ = oracle.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, s, r * K, K, bvh,
                                         sc.env_tf, sc.agent_tris, ref, par, n, nthreads=THREADS)
        st, pa = got[s]
        assert n == len(st)
        assert np.array_equal(st.view(np.uint64), ref[:n].view(np.uint64))
        assert np.array_equal(pa, par[:n])


def _c5_golden():
    import json

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config5_digests.json")) as f:
        return json.load(f)


def test_config5_256_joint(mpt_gpu, oracle):
    """The N = 1 north-star leg at the shape bench.py times it (`--seeds 256`, C5_WARMUP +
    C5_STEPS = 30 rounds of 4096 extensions): 256 wall-start blimp seeds in ONE step_many group
    from their start states -- every round a joint round (256 jobs dealt over the XCDs in the
    joint NN launch, one collide chunk of ~1 M units x 22 clusters split at the kernel's chunk
    boundary, the trees indexed from an empty cell tree inside the joint build and grown to ~110 k
    nodes each, ~28 M nodes in the last rounds' joint index).  Asserted:
    * the 256-seed digest equals that of eight separate 32-seed groups (what each GPU of eight
      runs, multiseed.shard_seeds) and the driver line's seeds_digest (tests/golden/
      config5_digests.json);
    * seeds 0 and 255 equal orc_engine_step's trees node for node (the reference's RRT::query
      loop, planners/rrt.hpp:42-94, batched), states and parents bitwise."""
    import hashlib
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from motionplanningtoolkit_amd import multiseed

    gold = _c5_golden()
    sc = scenes.blimp_scenario("all")
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, base, n = 4096, 1000, 256
    rounds = bench.C5_WARMUP + bench.C5_STEPS
    assert (rounds, K, base) == (gold["rounds"], gold["extensions_per_round"], gold["seed_base"])
    seeds = [base + i for i in range(n)]
    starts = {s: bench.seed_start(s, env, ag, mpt_gpu, "walls") for s in seeds}
    keep = (seeds[0], seeds[255])

    def grow(group_seeds):
        """per-tree digests of the group's seeds, and the kept seeds' trees"""
        engs = []
        for s in group_seeds:
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
            e.add_nodes(starts[s])
            e.set_nn("auto")
            engs.append(e)
        joint = torch.cuda.Stream()
        for _ in range(rounds):
            mpt_gpu.step_many(engs, K, [joint] * len(engs), joint)
        torch.cuda.synchronize()
        dig, trees, sizes = {}, {}, []
        for s, e in zip(group_seeds, engs):
            assert e.last_nn() == "tree"
            st, pa = e.read_tree(e.counters()["nodes"])
            dig[s] = multiseed.tree_digest(st, pa)
            sizes.append(len(st))
            if s in keep:
                trees[s] = (st, pa)
            e.close()
        mpt_gpu.joint_release(joint)
        return dig, trees, sizes

    def digest(d):
        return hashlib.sha256("".join(d[s] for s in sorted(d)).encode()).hexdigest()

    whole, trees, sizes = grow(seeds)
    assert min(sizes) > 10_000 and sum(sizes) > 20_000_000, (min(sizes), sum(sizes))
    assert digest(whole) == gold["seeds256"]
    shards = {}
    for r in range(8):
        shards.update(grow([seeds[i] for i in multiseed.shard_seeds(n, 8, r)])[0])
    assert shards == whole
    bvh = oracle.BVH(sc.env_tris)
    for s in keep:
        ref = np.zeros((1 + rounds * K, sc.dim))
        ref[0] = starts[s][0]
        par = np.zeros(1 + rounds * K, np.int32)
        m = 1
        for r in range(rounds):
            m, _, _ = oracle.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, s, r * K, K, bvh,
                                         sc.env_tf, sc.agent_tris, ref, par, m, nthreads=THREADS)
        st, pa = trees[s]
        assert m == len(st)
        assert np.array_equal(st.view(np.uint64), ref[:m].view(np.uint64))
        assert np.array_equal(pa, par[:m])
