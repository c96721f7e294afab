cd $GRAFT_REPO_ROOT
for cfg in "0 2" "1 2" "0 3" "1 3"; do set -- $cfg
  ENSVS_SPLITK=$1 ENSVS_STAGES_SMALL=$2 timeout -k 10 200 python -u tools/synth_probe.py 1 2>&1 | grep "B=" | sed "s/^/splitk=$1 stages=$2 /"
done
