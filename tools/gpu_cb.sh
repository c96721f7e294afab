# Multi-segment / accumulating plain bf16 GEMMs on hipBLASLt: SeparateF0 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/flag_ab.py --sf0 "BLAS:multi=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
