# round-4 call i: where block-max's overhead goes (8.8 M docs, per-wave layout from 64)
O=gpurun_out/round4_i; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
for a in 0 16384; do
  DI_WLONG_MIN=64 DI_PROFILE_ABLATE=$a SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_skew_a$a.json 2> $O/sweep_skew_a$a.err; fatal $? skew_$a; grep -q Traceback $O/sweep_skew_a$a.err && exit 1
  DI_WLONG_MIN=64 DI_PROFILE_ABLATE=$a SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 > $O/sweep_iid_a$a.json 2> $O/sweep_iid_a$a.err; fatal $? iid_$a; grep -q Traceback $O/sweep_iid_a$a.err && exit 1
done
DI_WLONG_MIN=64 DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 skew 1 > $O/phase_skew_bm1.txt 2>&1; fatal $? phase_bm
DI_WLONG_MIN=64 DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 skew 0 > $O/phase_skew_exh.txt 2>&1; fatal $? phase_exh
echo all-done
