# round-4 call g: the sparse-item batched scatter -- A/B of the retrieve legs against the
# previous build (tools/_old), index tests, 8.8 M skewed phases and block-max sweep
O=gpurun_out/round4_g; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_index.log 2>&1; rc=$?; tail -3 $O/pytest_index.log; fatal $rc index_tests
for v in old new old new; do
  if [ $v = old ]; then L="DEEPIMPACT_HIP_LIB=tools/_old/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1"; else L=""; fi
  env $L timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --steps 10 --warmup 2 --no-cpu > $O/ab_$v.$RANDOM.json 2>> $O/ab.err; fatal $? ab_$v
done
DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 skew 0 > $O/phase_skew_exh.txt 2>&1; fatal $? phase1
SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_bm.json 2> $O/sweep_bm.err; fatal $? sweep_bm
SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 > $O/sweep_bm_iid.json 2> $O/sweep_bm_iid.err; fatal $? sweep_bm_iid
echo all-done
