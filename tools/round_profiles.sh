# Round profile artifacts on the GPU box (run from the repo root):
#   gpurun -- 'bash tools/round_profiles.sh TAG'
#   gpurun_out/TAG_prof_train/   rocprofv3 --kernel-trace --stats of the bench's training line
#   gpurun_out/TAG_step_pmc.json HBM bytes per training step (FETCH_SIZE / WRITE_SIZE, separate
#                                passes over tools/step_pmc.py, tools/step_pmc_sum.py)
#   gpurun_out/TAG_gate_pmc.json the gate GEMM's HBM bytes per launch (tools/gate_gemm_pmc.py)
#   gpurun_out/TAG_prof_gate/    its kernel trace
# Every GPU step has its own time limit; the script stops at the first failure.
tag=${1:-rp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
o=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${tag}_prof_train -o train \
  -- python3 bench.py --no-synth --no-cpu-baseline --no-config2 --no-sf0 --no-census --no-shapes \
  --no-real-data --no-transformer --steps 8 > $o/${tag}_prof_train.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${tag}_pmc_fetch -o pmc \
  -- python3 tools/step_pmc.py > $o/${tag}_pmc_fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${tag}_pmc_write -o pmc \
  -- python3 tools/step_pmc.py > $o/${tag}_pmc_write.log 2>&1 || exit 3
python3 tools/step_pmc_sum.py $o/${tag}_pmc_fetch/pmc_counter_collection.csv \
  $o/${tag}_pmc_write/pmc_counter_collection.csv $o/${tag}_step_pmc.json > /dev/null || exit 4
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/${tag}_gpmc_fetch -o pmc \
  -- python3 tools/gate_gemm_pmc.py > $o/${tag}_gpmc_fetch.log 2>&1 || exit 5
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/${tag}_gpmc_write -o pmc \
  -- python3 tools/gate_gemm_pmc.py > $o/${tag}_gpmc_write.log 2>&1 || exit 6
python3 tools/pmc_summary.py $o/${tag}_gpmc_fetch/pmc_counter_collection.csv \
  $o/${tag}_gpmc_write/pmc_counter_collection.csv $o/${tag}_gate_pmc.json conv_gemm_b16_p8_kernel \
  > /dev/null || exit 7
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${tag}_prof_gate -o gate \
  -- python3 tools/gate_gemm_pmc.py > $o/${tag}_prof_gate.log 2>&1 || exit 8
echo "round profiles $tag done"
