# Iteration check on the GPU box (dev): all -m gpu tests, the gate-GEMM probe and the
# bench line without the CPU baseline.   gpurun -- 'bash tools/iter_run.sh'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/it_tests.log 2>&1 || { tail -30 gpurun_out/it_tests.log; exit 1; }
tail -1 gpurun_out/it_tests.log
timeout -k 10 120 python -u tools/gate_probe.py 20 > gpurun_out/it_gate.txt 2>&1 || exit 1
cat gpurun_out/it_gate.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/it_bench.json'))
s=d['synth']; r=d['roofline']
print('ms/step', round(d['ms_per_step'],2), 'gate us', round(r['launch_us'],1), 'frac', round(r['frac'],3), 'cfg2', round(d['config2']['ms_per_step'],2), 'IL', round(d['interaction_loss']['ms_per_step'],2))
print('pair acoustic ms', round(s['pair']['acoustic_ms'],1), 'rtf', round(s['pair']['rtf'],4), '6part', round(s['ensemble_6part']['rtf'],4), 'acoustic', round(s['ensemble_6part']['acoustic_ms'],1))
"
