# SeparateF0 schedule A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python tools/flag_ab.py --sf0 "acoustic_models.ENC_SIDE=0,acoustic_models.DEC_PREPACK=0" "acoustic_models.ENC_SIDE=0" "acoustic_models.DEC_PREPACK=0" > gpurun_out/cb_ab.txt 2>&1 || exit 3
