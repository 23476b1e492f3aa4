cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/hm_prof -o run --output-format csv -- python3 bench.py --env Humanoid-v2 --envs 1024 --hid 512,512,512 --steps 1 --warmup 1 --dtype bf16 --no-cpu-baseline > gpurun_out/hm_prof.log 2>&1 || exit 1
head -25 gpurun_out/hm_prof/run_kernel_stats.csv | cut -c1-160
