# sharded cooperative step counters vs HEAD's single counter (ENSVS_LIB A/B): benches and legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/ardec_bench.py > gpurun_out/cb_ardec_bench.txt 2>&1 || exit 3
ENSVS_LIB=ab/libensvs_HEAD.so timeout -k 10 300 python -u tools/ardec_bench.py >> gpurun_out/cb_ardec_bench.txt 2>&1 || exit 3
ENSVS_LIB=ab/libensvs_HEAD.so timeout -k 10 300 python -u tools/lstm_coop_bench.py > gpurun_out/cb_lstm_bench_old.txt 2>&1 || exit 2
timeout -k 10 300 python -u tools/lstm_coop_bench.py > gpurun_out/cb_lstm_bench.txt 2>&1 || exit 2
for r in 1 2; do
  timeout -k 10 300 python -u tools/flag_ab.py --sf0 "" >> gpurun_out/cb_ab.txt 2>&1 || exit 4
  ENSVS_LIB=ab/libensvs_HEAD.so timeout -k 10 300 python -u tools/flag_ab.py --sf0 "" | sed 's/^/HEAD /' >> gpurun_out/cb_ab.txt 2>&1 || exit 5
done
timeout -k 10 600 bash tools/lib_ab.sh ab/libensvs_HEAD.so >> gpurun_out/cb_ab.txt 2>&1 || exit 6
