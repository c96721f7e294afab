set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "" A B C; do
  if [ -n "$v" ]; then export ENSVS_LIB=$GRAFT_REPO_ROOT/build_var/lib$v.so; fi
  echo "== variant [$v]" >> gpurun_out/r4_lstm_var.txt
  timeout -k 10 120 python3 -u tools/lstm_mfma_bench.py >> gpurun_out/r4_lstm_var.txt 2>&1 || exit 1
done
