# hipBLASLt grids with and without TENSILE_STREAMK_DATA_PARALLEL (kernel traces)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/blasp0 -o b -- python3 tools/blas_probe.py > gpurun_out/blasp0.log 2>&1 || exit 1
TENSILE_STREAMK_DATA_PARALLEL=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/blasp1 -o b -- python3 tools/blas_probe.py > gpurun_out/blasp1.log 2>&1 || exit 2
