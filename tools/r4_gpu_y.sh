set -o pipefail
cd $GRAFT_REPO_ROOT
for L in "" build_var/libensvs_nt.so; do
echo "== lib=[$L]" >> gpurun_out/r4_nt_probe.txt
ENSVS_LIB=$L timeout -k 10 200 python3 -u tools/dgrad_probe.py 2>&1 | grep -v amdgpu >> gpurun_out/r4_nt_probe.txt || exit 1
done
