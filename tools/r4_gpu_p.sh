set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "" build_var/libensvs_noSMX.so build_var/libensvs_noSMB.so build_var/libensvs_noTG2.so build_var/libensvs_noVEC4.so; do
  ENSVS_LIB=$L timeout -k 10 200 python3 -u -m pytest -m gpu -q --timeout 150 --timeout-method thread tests/test_transformer.py -k "large_t or dropout" > gpurun_out/r4_p.log 2>&1
  echo "lib=[$L] rc=$? $(tail -1 gpurun_out/r4_p.log)" >> gpurun_out/r4_p_sum.txt
done
