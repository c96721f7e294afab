# Re-check of two C-ABI routing switches after this round's changes: step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u tools/flag_ab.py "BLAS:min_rows=1" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
