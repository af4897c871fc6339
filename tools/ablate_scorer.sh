# Profiling helper: time score_blocks with phases skipped (DI_PROFILE_ABLATE bit0 = no
# scatter, bit1 = no selection) and one encode bench.  Not a test; results are wrong by design.
set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2 3; do
  DI_PROFILE_ABLATE=$a timeout -k 10 300 python bench.py --legs retrieve --steps 5 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate $a', d['retrieve']['kernel_ms'])" || exit 1
done
timeout -k 10 300 python bench.py --legs encode --steps 5 --warmup 1 --no-cpu > gpurun_out/enc.json 2>/dev/null && python3 -c "
import json; d=json.load(open('gpurun_out/enc.json')); print(d['value'], {k: round(v['ms_per_step'],2) for k,v in d['encode']['kernels'].items()}, d['encode']['gemm_tflops'])"
