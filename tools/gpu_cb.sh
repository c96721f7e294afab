# BF16_ACT min_reuse 1: second main-line A/B and SeparateF0 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u tools/flag_ab.py "BF16_ACT:min_reuse=1" "" > gpurun_out/cb_ab2.txt 2>&1 || exit 3
timeout -k 10 900 python -u tools/flag_ab.py --sf0 "BF16_ACT:min_reuse=1" "" > gpurun_out/cb_ab3.txt 2>&1 || exit 4
