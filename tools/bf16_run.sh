set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_pipeline.py tests/test_gpu_iteration.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bf16_t2.log 2>&1 || { tail -40 gpurun_out/bf16_t2.log; exit 1; }
tail -3 gpurun_out/bf16_t2.log
timeout -k 10 300 python bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/bf16_bench_hopper.json 2> gpurun_out/bf16_bench_hopper.err || { tail gpurun_out/bf16_bench_hopper.err; exit 1; }
cat gpurun_out/bf16_bench_hopper.json
timeout -k 10 300 python bench.py --env CartPole-v0 --dtype bf16 --steps 5 --no-cpu-baseline > gpurun_out/bf16_bench_cartpole.json 2> gpurun_out/bf16_bench_cartpole.err || { tail gpurun_out/bf16_bench_cartpole.err; exit 1; }
cat gpurun_out/bf16_bench_cartpole.json
timeout -k 10 400 python bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 3 --warmup 1 --dtype bf16 --no-cpu-baseline > gpurun_out/bf16_bench_humanoid.json 2> gpurun_out/bf16_bench_humanoid.err || { tail gpurun_out/bf16_bench_humanoid.err; exit 1; }
cat gpurun_out/bf16_bench_humanoid.json
