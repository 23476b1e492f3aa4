set -o pipefail
cd $GRAFT_REPO_ROOT
for B in 64 0 64 0; do
  MRL_VF_SIDE_COPY_BLOCKS=$B timeout -k 10 200 python bench.py --steps 20 > gpurun_out/ab_$B.json 2>gpurun_out/ab_$B.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_$B.json').read().strip().splitlines()[-1]);print($B,d['ms_per_step'],d['phase_ms_per_iter'])"
done
