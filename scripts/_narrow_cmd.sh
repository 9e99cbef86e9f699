set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_collide_gpu.py > gpurun_out/narrow_tests.log 2>&1 && tail -3 gpurun_out/narrow_tests.log &&
BENCH_ARGS="--workload blimp-room --steps 30 --warmup 5 --no-cpu" bash scripts/ab.sh narrow_room "base:" "glob:MPT_NARROW_LDS=0" &&
BENCH_ARGS="--steps 30 --warmup 5 --no-cpu" bash scripts/ab.sh narrow_c2 "base:" "glob:MPT_NARROW_LDS=0"
