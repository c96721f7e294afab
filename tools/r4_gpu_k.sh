set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for L in ab/base/ensemble_svs_with_interactions_amd/libensvs.so build_var/libensvs_d0i0.so build_var/libensvs_d0i1.so build_var/libensvs_d1i0.so build_var/libensvs_d1i1.so build_var/libensvs_d2i0.so; do
  echo "== $L" >> gpurun_out/r4_lstm_var_k.txt
  ENSVS_LIB=$L timeout -k 10 120 python3 -u tools/lstm_mfma_bench.py 2>/dev/null | grep mfma >> gpurun_out/r4_lstm_var_k.txt || exit 1
done
done
