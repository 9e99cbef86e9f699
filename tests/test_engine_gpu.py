"""GPU parity: one batched RRT round of the device engine (k_sample -> k_knn1 -> k_steer ->
k_collide -> ordered append) checked stage by stage against the oracle.

Bars: every stage is bit-exact -- samples, NN ids, steered states and poses, collision
verdicts and the append order.  The blimp / snake steering's sin / cos / tan are the
correctly rounded values on both sides (fcl_math.h cr_*, oracle orc_cr_*; DESIGN.md §2 on
why the engine contract is not the host libm)."""
import math

import numpy as np
import pytest

from motionplanningtoolkit_amd import scenes

pytestmark = pytest.mark.gpu

def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def make(mpt, sc, n0, K, seed, cap_extra=None):
    rng = np.random.default_rng(seed)
    tree = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    ag = mpt.AgentMesh(sc.agent_tris)
    eng = mpt.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt,
                        capacity=n0 + (cap_extra if cap_extra is not None else 4 * K), seed=seed)
    eng.add_nodes(tree)
    return eng, tree


def expected_controls(oracle, sc, seed, g):
    if sc.kind == 0:
        return [oracle.engine_uniform(seed, g * 64 + 32 + j, -1.0, 1.0) for j in range(3)]
    if sc.kind == 1:
        return [oracle.engine_uniform(seed, g * 64 + 32, -1, 1), oracle.engine_uniform(seed, g * 64 + 33, -0.1745, 0.1745),
                oracle.engine_uniform(seed, g * 64 + 34, -1, 1)]
    return [oracle.engine_uniform(seed, g * 64 + 32, -0.1, 1), oracle.engine_uniform(seed, g * 64 + 33, -math.pi / 18,
                                                                                     math.pi / 18)]


def check_round(mpt, oracle, sc, eng, tree, seed, ext_base, K):
    eng.step(K)
    samples, nn, ends, verdict = eng.last_round(K)
    poses, pcount = eng.last_poses(K)
    inf = eng.info()
    # 1. samples: pure +,-,* arithmetic on the counter hash -> bit-exact
    exp_s = np.array([[oracle.engine_uniform(seed, (ext_base + k) * 64 + j, lo, hi)
                       for j, (lo, hi) in enumerate(sc.ranges)] for k in range(K)])
    assert np.array_equal(bits(samples), bits(exp_s))
    # 2. nearest neighbours over the snapshot
    ri, _ = oracle.knn(tree, samples, 1)
    assert np.array_equal(nn, ri[:, 0])
    # 3. steer + poses (correctly rounded trig on both sides: bit-exact)
    exp_end = np.zeros_like(ends)
    for k in range(K):
        g = ext_base + k
        frm = tree[nn[k] - 1]
        c = expected_controls(oracle, sc, seed, g)
        if sc.kind == 0:
            r = np.array(c)
            dist = math.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2])
            exp_end[k] = frm + r / dist
            exp_p = oracle.omni_get_poses(frm, exp_end[k], sc.cc_dt)
            assert pcount[k] == len(exp_p)
            assert np.array_equal(bits(ends[k]), bits(exp_end[k]))  # no transcendentals
            assert np.array_equal(bits(poses[k, :pcount[k], 0]), bits(exp_p))
        elif sc.kind == 1:
            exp_end[k] = oracle.blimp_do_step(sc.prm, frm, c[0], c[1], c[2], sc.steer_dt, trig="cr")
            exp_p = oracle.blimp_get_poses(sc.prm, frm, c, sc.steer_dt, sc.cc_dt, trig="cr")
            assert pcount[k] == len(exp_p)
            assert np.array_equal(bits(poses[k, :pcount[k], 0]), bits(exp_p))
        else:
            exp_end[k] = oracle.snake_do_step(sc.prm, frm, c[0], c[1], sc.steer_dt, trig="cr")
            exp_p = oracle.snake_get_poses(sc.prm, frm, c, sc.steer_dt, sc.cc_dt, trig="cr")
            assert pcount[k] == len(exp_p)
            assert np.array_equal(bits(poses[k, :pcount[k]]), bits(exp_p))
    assert np.array_equal(bits(ends), bits(exp_end))
    # 4. verdicts on the device's own poses: bit-exact
    flat = np.concatenate([poses[k, :pcount[k]] for k in range(K)]).reshape(-1, inf["links"], 12)
    off = np.r_[0, np.cumsum(pcount)]
    ref_v = oracle.collide_batch(sc.env_tris, sc.env_tf, [sc.agent_tris] * inf["links"], flat, off)
    assert np.array_equal(verdict, ref_v)
    # 5. ordered append
    valid = np.nonzero(verdict == 0)[0]
    n_new = len(tree) + len(valid)
    c = eng.counters()
    assert c["nodes"] == n_new and c["valid"] >= len(valid)
    t2, par = eng.read_tree(n_new)
    assert np.array_equal(bits(t2[:len(tree)]), bits(tree))
    assert np.array_equal(bits(t2[len(tree):]), bits(ends[valid]))
    assert np.array_equal(par[len(tree):], nn[valid])
    return t2, verdict


@pytest.mark.parametrize("nn_mode", ["brute", "grid", "tree"])
@pytest.mark.parametrize("name", ["omni", "blimp", "snake"])
def test_engine_rounds(mpt_gpu, oracle, name, nn_mode):
    if name == "omni":
        sc, n0, K = scenes.omni_scenario(), 3000, 1024
    elif name == "blimp":
        sc, n0, K = scenes.blimp_scenario("all"), 5000, 1500
    else:
        sc, n0, K = scenes.snake_scenario("corridor"), 3000, 700
    seed = 1234
    eng, tree = make(mpt_gpu, sc, n0, K, seed)
    eng.set_nn(nn_mode)
    tree, v1 = check_round(mpt_gpu, oracle, sc, eng, tree, seed, 0, K)
    assert 0 < v1.sum() < K or name == "snake"
    # second round sees the first round's nodes
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, seed, K, K // 2 + 3)


@pytest.mark.parametrize("K", [2048, 6144])
def test_engine_tree_nn_large_blob(mpt_gpu, oracle, K):
    """Cell-tree NN (config 5's index, cell_tree.hip) over a 40k-node RRT-like blob: the first
    round's full build (hipcub sort of every code, buckets of <= 8 points, a directory of
    several thousand entries and box levels up to the root); the second round's build is
    incremental: K = 6144 new points, so the chunked sort ranks across more than 8 chunks of
    512, many buckets split, and the directory merge places entries across workgroups."""
    sc = scenes.blimp_scenario("all")
    rng = np.random.default_rng(77)
    n0 = 40_000
    tree = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    tree[:, :3] = np.array([88.6, 68.9, 57.1]) + rng.normal(0.0, 6.0, size=(n0, 3))
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    eng = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, capacity=n0 + 4 * K,
                            seed=4242)
    eng.add_nodes(tree)
    eng.set_nn("tree")
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 4242, 0, K)
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 4242, K, K)


def test_cell_tree_duplicates_truncation_bulk_and_overgrowth(mpt_gpu, oracle):
    """The incremental cell tree (cell_tree.hip) through its edge cases, every round checked
    stage by stage against the oracle: a full build over a blob holding 40 and 20 copies of two
    states (equal codes, more than a bucket holds: grouped by row); incremental rounds that
    append to and split buckets; a truncation (set_size: the next build starts over); a bulk
    add_nodes of more copies; a round of K = 9000 (more new points than one round inserts, so the
    next build is a full one); and the index error counter stays clear."""
    sc = scenes.blimp_scenario("all")
    rng = np.random.default_rng(5)
    blob = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(3000, sc.dim))
    blob[:, :3] = np.array([40.0, 60.0, 50.0]) + rng.normal(0.0, 4.0, size=(3000, 3))
    dup_a, dup_b = blob[7].copy(), blob[1234].copy()
    tree = np.concatenate([blob, np.tile(dup_a, (40, 1)), np.tile(dup_b, (20, 1))])
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    eng = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, capacity=40_000, seed=99)
    eng.add_nodes(tree)
    eng.set_nn("tree")
    base = 0
    for K in (1024, 1024):
        tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 99, base, K)
        base += K
    eng.set_size(2500)
    tree = tree[:2500]
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 99, base, 700)
    base += 700
    more = np.concatenate([np.tile(dup_b, (30, 1)), rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(500, sc.dim))])
    eng.add_nodes(more)
    tree = np.concatenate([tree, more])
    for K in (1024, 9000, 512):
        tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 99, base, K)
        base += K
    assert eng.last_nn() == "tree"
    assert eng.counters()["nodes"] == len(tree)


@pytest.mark.parametrize("name", ["omni", "blimp"])
def test_engine_grid_blob_and_sparse(mpt_gpu, oracle, name):
    """The grid 1-NN (bucketed run kernel) on a tree that is half a tight blob and half
    sparse: the blob's few cells hold thousands of points each (one run spreads them over the
    group's lanes for many steps), and in the sparse half the first pass often does not settle
    a query (the walk continues with ring 2 and beyond).  NN ids and the whole round stay
    bit-exact against the oracle."""
    sc = scenes.blimp_scenario("all") if name == "blimp" else scenes.omni_scenario()
    rng = np.random.default_rng(99)
    n0, K = 6000, 4096
    tree = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    ctr = 0.5 * (sc.ranges[:3, 0] + sc.ranges[:3, 1])
    tree[: n0 // 2, :3] = ctr + rng.normal(0.0, 0.01 * (sc.ranges[0, 1] - sc.ranges[0, 0]), size=(n0 // 2, 3))
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    eng = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, capacity=n0 + 4 * K,
                            seed=31)
    eng.add_nodes(tree)
    eng.set_nn("grid")
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 31, 0, K)
    tree, _ = check_round(mpt_gpu, oracle, sc, eng, tree, 31, K, K // 2 + 5)
    assert eng.last_nn() == "grid"


def test_engine_round_with_pair_overflow(mpt_gpu, oracle):
    """The blimp against the blimp mesh itself as the environment, every pose within a few
    units of it: clusters overlap far more env triangles than a pair segment holds, so units
    overflow and k_narrow's last workgroups re-run them whole with the fused walk.  The round
    must still match the oracle stage by stage, and the counters must show the re-runs."""
    import dataclasses

    base = scenes.blimp_scenario("all")
    ranges = base.ranges.copy()
    ranges[:3] = [-3.0, 3.0]
    sc = dataclasses.replace(base, env_tris=base.agent_tris.copy(), env_tf=scenes.IDENTITY_TF.copy(), ranges=ranges)
    seed, n0, K = 4321, 500, 256
    eng, tree = make(mpt_gpu, sc, n0, K, seed)
    eng.set_nn("brute")
    eng.collide_stats(True)
    _, v = check_round(mpt_gpu, oracle, sc, eng, tree, seed, 0, K)
    st = eng.collide_stats(False)
    assert st["fused_reruns"] > 0
    assert v.sum() > 0


def test_joint_rounds_with_pair_overflow(mpt_gpu):
    """The overflow scene above in joint rounds: the joint collide's overflowed units are
    re-run inside the joint append launch (k_append_jobs takes k_overflow's work, and its last
    block appends every engine's extensions in order).  Three engines must grow exactly the
    trees they grow alone, where the solo rounds count their fused re-runs."""
    import dataclasses

    import torch

    base = scenes.blimp_scenario("all")
    ranges = base.ranges.copy()
    ranges[:3] = [-3.0, 3.0]
    sc = dataclasses.replace(base, env_tris=base.agent_tris.copy(), env_tf=scenes.IDENTITY_TF.copy(), ranges=ranges)
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, seeds, n0 = 256, 3, (71, 72, 73), 300

    def grow(joint):
        engs = []
        for s in seeds:
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, n0 + rounds * K, s)
            e.add_nodes(np.random.default_rng(s).uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim)))
            e.set_nn("tree")
            engs.append(e)
        reruns = 0
        js = torch.cuda.Stream()
        for _ in range(rounds):
            if joint:
                mpt_gpu.step_many(engs, K, [js] * len(engs), js)
            else:
                for e in engs:
                    e.collide_stats(True)
                    e.step(K)
                    reruns += e.collide_stats(False)["fused_reruns"]
        torch.cuda.synchronize()
        out = [e.read_tree(e.counters()["nodes"]) for e in engs]
        if joint:
            mpt_gpu.joint_release(js)
        return out, reruns

    solo, reruns = grow(False)
    joint, _ = grow(True)
    assert reruns > 0
    for (sa, pa), (sb, pb) in zip(solo, joint):
        assert np.array_equal(bits(sa), bits(sb))
        assert np.array_equal(pa, pb)


@pytest.mark.parametrize("name", ["omni", "blimp", "snake"])
def test_engine_rounds_fused_collide(mpt_gpu, oracle, name):
    """The same stage-by-stage parity with the fused collision kernel in the round."""
    if name == "omni":
        sc, n0, K = scenes.omni_scenario(), 2000, 800
    elif name == "blimp":
        sc, n0, K = scenes.blimp_scenario("all"), 3000, 1200
    else:
        sc, n0, K = scenes.snake_scenario("corridor"), 2000, 500
    mpt_gpu.set_collide_mode("fused")
    try:
        eng, tree = make(mpt_gpu, sc, n0, K, 99)
        eng.set_nn("grid")
        check_round(mpt_gpu, oracle, sc, eng, tree, 99, 0, K)
    finally:
        mpt_gpu.set_collide_mode("split")


def test_engine_grid_equals_brute_over_growing_rounds(mpt_gpu, oracle):
    """A growing tree (no reset) over several rounds: the grid and the brute-force NN
    engines must build the same tree bit for bit (rounds build the grid from scratch)."""
    sc = scenes.blimp_scenario("last")
    trees = []
    for mode in ("brute", "grid", "tree"):
        eng, tree = make(mpt_gpu, sc, 6000, 4096, 77, cap_extra=5 * 4096)
        eng.set_nn(mode)
        for K in (4096, 1000, 4096, 333, 2048):
            eng.step(K)
        n = eng.counters()["nodes"]
        trees.append(eng.read_tree(n))
    for t in trees[1:]:
        assert np.array_equal(bits(trees[0][0]), bits(t[0]))
        assert np.array_equal(trees[0][1], t[1])


@pytest.mark.parametrize("nn_mode", ["grid", "tree"])
@pytest.mark.parametrize("name", ["blimp", "snake"])
def test_engine_trees_equal_oracle_over_rounds(mpt_gpu, oracle, name, nn_mode):
    """Whole trees, not stages: several rounds grown on the device (each round sees the
    previous rounds' nodes) equal the oracle's engine rounds (orc_engine_step: kd-tree NN,
    correctly rounded steering trig, AABB-tree + FCL SAT collision) node for node, states and
    parents bitwise."""
    if name == "blimp":
        sc, n0, Ks = scenes.blimp_scenario("all"), 5000, (2048, 777, 2048)
    else:
        sc, n0, Ks = scenes.snake_scenario("corridor"), 5000, (1024, 333, 1024)
    seed = 4242
    eng, tree = make(mpt_gpu, sc, n0, max(Ks), seed, cap_extra=sum(Ks))
    eng.set_nn(nn_mode)
    for K in Ks:
        eng.step(K)
    n = eng.counters()["nodes"]
    got, gpar = eng.read_tree(n)
    ref = np.zeros((n0 + sum(Ks), sc.dim))
    ref[:n0] = tree
    rpar = np.zeros(n0 + sum(Ks), np.int32)
    bvh = oracle.BVH(sc.env_tris)
    m, base = n0, 0
    for K in Ks:
        m, _, _ = oracle.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, seed, base, K, bvh,
                                     sc.env_tf, sc.agent_tris, ref, rpar, m, nthreads=8)
        base += K
    assert m == n and n > n0
    assert np.array_equal(bits(got), bits(ref[:n]))
    assert np.array_equal(gpar[n0:], rpar[n0:n])


@pytest.mark.parametrize("name", ["blimp", "snake"])
def test_engine_tree_from_one_root(mpt_gpu, name):
    """A tree grown from a single root (the RRT case: nodes clustered around the start,
    samples all over the sampling box): the Morton-tree and brute-force NN engines build the
    same tree bit for bit."""
    if name == "blimp":
        sc, root = scenes.blimp_scenario("all"), np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    else:
        sc = scenes.snake_scenario("corridor")
        root = np.asarray(sc.start, np.float64).reshape(1, -1)
    trees = []
    for mode in ("brute", "tree", "auto"):
        env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
        ag = mpt_gpu.AgentMesh(sc.agent_tris)
        eng = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + 8 * 2048, 5)
        eng.add_nodes(root)
        eng.set_nn(mode)
        for _ in range(8):
            eng.step(2048)
        n = eng.counters()["nodes"]
        trees.append(eng.read_tree(n))
    assert len(trees[0][0]) > 100
    for t in trees[1:]:
        assert np.array_equal(bits(trees[0][0]), bits(t[0]))
        assert np.array_equal(trees[0][1], t[1])


def test_engines_on_streams_match_one_stream(mpt_gpu):
    """Config 5's execution model: many independent seeds, each its own engine grown from one
    root, their rounds interleaved over several HIP streams (first-use allocations happen
    while other engines' kernels run).  Every seed's tree must equal the one it grows alone
    on the default stream, bit for bit."""
    import torch

    sc = scenes.blimp_scenario("all")
    root = np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, seeds = 2048, 5, list(range(300, 312))

    def grow(streams):
        engs = []
        for s in seeds:
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
            e.add_nodes(root)
            engs.append(e)
        for _ in range(rounds):
            for j, e in enumerate(engs):
                e.step(K, streams[j % len(streams)] if streams else None)
        torch.cuda.synchronize()
        out = []
        for e in engs:
            n = e.counters()["nodes"]
            out.append(e.read_tree(n))
            e.close()
        return out

    alone = grow(None)
    mixed = grow([torch.cuda.Stream() for _ in range(4)])
    for (sa, pa), (sb, pb) in zip(alone, mixed):
        assert len(sa) > 1
        assert np.array_equal(bits(sa), bits(sb)) and np.array_equal(pa, pb)


def test_step_many_matches_single_steps(mpt_gpu, oracle):
    """mpt_rrt_step_many (config 5's joint NN launch): twelve seeds over four streams, all but
    one on the cell tree (one launch of k_ct_nn1_jobs per round) and one on the grid (its
    own query), must grow exactly the trees each seed grows alone with mpt_rrt_step -- and, for
    three of the seeds, exactly the oracle's engine rounds (orc_engine_step) from the same
    root."""
    import torch

    sc = scenes.blimp_scenario("all")
    root = np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, seeds = 2048, 4, list(range(500, 512))
    modes = ["tree"] * (len(seeds) - 1) + ["grid"]

    def grow(joint):
        engs = []
        for s, m in zip(seeds, modes):
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
            e.add_nodes(root)
            e.set_nn(m)
            engs.append(e)
        streams = [torch.cuda.Stream() for _ in range(4)]
        for _ in range(rounds):
            if joint:
                mpt_gpu.step_many(engs, K, [streams[j % 4] for j in range(len(engs))], torch.cuda.Stream())
            else:
                for e in engs:
                    e.step(K)
        torch.cuda.synchronize()
        out = []
        for e in engs:
            assert e.last_nn() == modes[len(out)]
            out.append(e.read_tree(e.counters()["nodes"]))
            e.close()
        return out

    alone = grow(False)
    joint = grow(True)
    for (sa, pa), (sb, pb) in zip(alone, joint):
        assert len(sa) > 2048
        assert np.array_equal(bits(sa), bits(sb)) and np.array_equal(pa, pb)
    bvh = oracle.BVH(sc.env_tris)
    for j in (0, 5, len(seeds) - 1):
        ref = np.zeros((1 + rounds * K, sc.dim))
        ref[0] = root[0]
        par = np.zeros(1 + rounds * K, np.int32)
        n = 1
        for r in range(rounds):
            n, _, _ = oracle.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, seeds[j], r * K, K, bvh,
                                         sc.env_tf, sc.agent_tris, ref, par, n, nthreads=8)
        sb, pb = joint[j]
        assert n == len(sb)
        assert np.array_equal(bits(sb), bits(ref[:n])) and np.array_equal(pb, par[:n])


def test_step_many_groups_on_separate_joint_streams(mpt_gpu):
    """Several step_many groups issued back to back from one host thread, each group on its own
    engine streams and its own joint stream (bench.py --joint-groups): the joint job tables and
    sort buffers belong to the joint stream, so one group's staging never overwrites what
    another group's build and NN kernels still read (the round-1 race).  Group A: blimp seeds of
    ragged sizes (one root; 3 000, 9 000 and 140 000 pre-added nodes: several bbox workgroups,
    the box-level ticket path, more than 131 072 points); group B: blimp seeds from one root;
    group C: the snake (d = 15, the 16-wide register rows).  Every tree must equal the one its
    seed grows alone with mpt_rrt_step, bit for bit; the joint build / NN times are reported
    per joint stream."""
    import torch

    blimp = scenes.blimp_scenario("all")
    snake = scenes.snake_scenario("corridor")
    root_b = np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    rng = np.random.default_rng(21)

    def blob(n):
        t = rng.uniform(blimp.ranges[:, 0], blimp.ranges[:, 1], size=(n, 7))
        t[:, :3] = root_b[0, :3] + rng.normal(0.0, 8.0, size=(n, 3))
        return t

    K, rounds = 2048, 3
    specs = []  # (scenario, seed, initial nodes, group)
    for s, n in zip(range(700, 704), (1, 3000, 9000, 140_000)):
        specs.append((blimp, s, root_b if n == 1 else blob(n), 0))
    for s in range(710, 714):
        specs.append((blimp, s, root_b, 1))
    for s in range(720, 724):
        specs.append((snake, s, np.asarray(snake.start, np.float64).reshape(1, -1), 2))
    handles = {}
    for sc in (blimp, snake):
        handles[sc.name] = (mpt_gpu.Environment(sc.env_tris, sc.env_tf), mpt_gpu.AgentMesh(sc.agent_tris))
    groups = [[j for j, sp in enumerate(specs) if sp[3] == g] for g in range(3)]

    def grow(joint):
        engs = []
        for sc, s, init, _ in specs:
            env, ag = handles[sc.name]
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, len(init) + rounds * K, s)
            e.add_nodes(init)
            e.set_nn("tree")
            engs.append(e)
        streams = [[torch.cuda.Stream() for _ in range(2)] for _ in groups]
        joints = [torch.cuda.Stream() for _ in groups]
        times = None
        for r in range(rounds):
            if joint:
                if r == rounds - 1:
                    engs[groups[0][0]].enable_timing(True)
                for g, idx in enumerate(groups):
                    mpt_gpu.step_many([engs[j] for j in idx], K, [streams[g][k % 2] for k in range(len(idx))], joints[g])
            else:
                for e in engs:
                    e.step(K)
        torch.cuda.synchronize()
        if joint:
            times = mpt_gpu.joint_times(joints[0])
        out = []
        for e in engs:
            assert e.last_nn() == "tree"
            out.append(e.read_tree(e.counters()["nodes"]))
            e.close()
        return out, times

    alone, _ = grow(False)
    joint, times = grow(True)
    for (sa, pa), (sb, pb) in zip(alone, joint):
        assert len(sa) > K
        assert np.array_equal(bits(sa), bits(sb)) and np.array_equal(pa, pb)
    assert times["build"] > 0 and times["nn"] > 0


def test_engine_set_size_and_capacity(mpt_gpu, oracle):
    sc = scenes.omni_scenario()
    eng, tree = make(mpt_gpu, sc, 100, 256, 5, cap_extra=50)
    eng.step(256)
    c = eng.counters()
    assert c["nodes"] == 150 and c["capacity_drops"] > 0
    eng.set_size(100)
    assert eng.counters()["nodes"] == 100
    t, _ = eng.read_tree(100)
    assert np.array_equal(t, tree)


def test_joint_round_matches_single_steps(mpt_gpu):
    """mpt_rrt_step_many as a joint round (every engine on the Morton tree, one launch per stage
    for all of them, engine j's round buffers at offset j * K of the joint state): six blimp
    seeds, one of them truncated with set_size between rounds (applied by the joint sample
    launch; the index then rebuilds from scratch), must grow exactly the trees each seed grows
    alone, and an engine's last-round intermediates (samples, NN ids, end states, verdicts,
    poses) must equal its solo round's."""
    import torch

    sc = scenes.blimp_scenario("all")
    root = np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, seeds = 1024, 5, list(range(900, 906))

    def grow(joint):
        engs = []
        for s in seeds:
            e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
            e.add_nodes(root)
            e.set_nn("tree")
            engs.append(e)
        streams = [torch.cuda.Stream() for _ in range(3)]
        js = torch.cuda.Stream()
        for r in range(rounds):
            if r == 3:
                engs[2].set_size(500)
            if joint:
                engs[0].enable_timing(r == rounds - 1)
                mpt_gpu.step_many(engs, K, [streams[j % 3] for j in range(len(engs))], js)
            else:
                for e in engs:
                    e.step(K)
        torch.cuda.synchronize()
        times = mpt_gpu.joint_stage_times(js) if joint else None
        out = []
        for e in engs:
            assert e.last_nn() == "tree"
            out.append((e.read_tree(e.counters()["nodes"]), e.last_round(K), e.last_poses(K)))
        if joint:
            # a joint round's stage times live on the joint stream, not in the engine's ring
            with pytest.raises(mpt_gpu.MptError):
                engs[0].kernel_times()
            mpt_gpu.joint_release(js)
            # the slices an engine's last round points into are gone with the joint state
            with pytest.raises(mpt_gpu.MptError):
                engs[1].last_round(K)
            with pytest.raises(mpt_gpu.MptError):
                engs[1].last_poses(K)
        for e in engs:
            e.close()
        return out, times

    alone, _ = grow(False)
    joint, times = grow(True)
    for (ta, ra, pa), (tb, rb, pb) in zip(alone, joint):
        assert len(ta[0]) > K
        assert np.array_equal(bits(ta[0]), bits(tb[0])) and np.array_equal(ta[1], tb[1])
        for x, y in zip(ra, rb):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
        assert np.array_equal(bits(pa[0]), bits(pb[0])) and np.array_equal(pa[1], pb[1])
    assert set(times) == {"sample", "nn_build", "nn_query", "steer", "collide", "append"}
    assert all(v > 0 for v in times.values())


def test_joint_nn_xcd_mappings_same_ids(mpt_gpu, oracle):
    """The joint NN launch under every XCD mapping (k_ct_nn1_jobs parts: 0 = each tree's
    workgroups over all eight XCDs, P = 1, 2, 4, 8 = each tree in P contiguous runs, one XCD
    each; mpt_rrt_joint_replay_nn) writes the same ids and squared distances -- which workgroup
    answers a query changes nothing -- and they are the exact 1-NN of the oracle's kd-tree over
    the index the round queried (flannkdtreewrapper.hpp:57-89)."""
    import torch

    sc = scenes.blimp_scenario("all")
    root = np.array([[88.6, 68.9, 57.1, 0, 0, 0, 0.0]])
    env = mpt_gpu.Environment(sc.env_tris, sc.env_tf)
    ag = mpt_gpu.AgentMesh(sc.agent_tris)
    K, rounds, n = 1024, 4, 16
    engs = []
    for s in range(700, 700 + n):
        e = mpt_gpu.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + rounds * K, s)
        e.add_nodes(root)
        e.set_nn("tree")
        engs.append(e)
    js = torch.cuda.Stream()
    sizes = []
    for r in range(rounds):
        if r == rounds - 1:
            torch.cuda.synchronize()
            sizes = [e.counters()["nodes"] for e in engs]  # the last round's index
        mpt_gpu.step_many(engs, K, [js] * n, js)
    torch.cuda.synchronize()
    base = [e.last_round(K) for e in engs]
    for parts in (0, 1, 2, 4, 8, 0):
        mpt_gpu.joint_replay_nn(js, parts)
        torch.cuda.synchronize()
        for e, b in zip(engs, base):
            assert np.array_equal(e.last_round(K)[1], b[1]), parts
    with pytest.raises(mpt_gpu.MptError):
        mpt_gpu.joint_replay_nn(js, 3)  # a tree's 1024 workgroups do not split into 3 runs
    for j in (0, n - 1):
        tree, _ = engs[j].read_tree(sizes[j])
        ref, _ = oracle.KDTree(tree).knn(base[j][0], 1)
        assert np.array_equal(base[j][1], ref[:, 0])
    for e in engs:
        e.close()
    mpt_gpu.joint_release(js)
