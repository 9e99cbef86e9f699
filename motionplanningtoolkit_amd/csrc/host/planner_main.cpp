// planner_main.cpp -- `mpt_planner <file.inst>`: the reference's CLI (main.cpp:192-212) on the
// GPU path.  Optional build keys: `Max Iterations ? N` (RRT::query iterationsAtATime).
#include <cstdio>
#include <exception>
#include <string>

#include "compose.hpp"

int main(int argc, char *argv[]) {
    if (argc < 2) {
        fprintf(stderr, "no instance file provided!\n");
        return 1;
    }
    try {
        if (mpt_init(0) != MPT_OK) {
            fprintf(stderr, "mpt_init: %s\n", mpt_last_error());
            return 2;
        }
        mpt_host::InstanceFileMap args(argv[1]);
        if (args.exists("Batch Size")) {  // batched throughput mode (compose.hpp run_batched)
            const auto r = mpt_host::run_batched_inst(argv[1]);
            int64_t solved = 0, nodes = 0;
            for (size_t i = 0; i < r.nodes.size(); ++i) {
                solved += r.solved[i];
                nodes += r.nodes[i];
            }
            fprintf(stdout, "RRT batched: %zu trees, %lld rounds, %lld extensions checked, %lld valid, %.3f s, "
                    "%.1f M valid ext/s, %lld nodes, %lld trees reached the goal\n",
                    r.nodes.size(), (long long)r.rounds, (long long)r.checked, (long long)r.valid, r.seconds,
                    r.seconds > 0 ? r.valid / r.seconds / 1e6 : 0.0, (long long)nodes, (long long)solved);
            return 0;
        }
        const int iters = std::stoi(args.value_or("Max Iterations", "-1"));
        const auto r = mpt_host::run_inst(argv[1], iters);
        fprintf(stderr, "tree edges: %zu solved: %d\n", r.dim ? r.ends.size() / r.dim : 0, r.solved ? 1 : 0);
    } catch (const std::exception &e) {
        fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
