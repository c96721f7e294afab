# Reverse-diffusion iteration check (dev): GPU tests, then a kernel trace of the pair
# inference probe reduced to kernel time vs launch gaps per diffusion step, then the bench.
#   gpurun -- 'bash tools/synth_iter.sh'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/si_tests.log 2>&1 || { tail -40 gpurun_out/si_tests.log; exit 1; }
tail -1 gpurun_out/si_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/si_prof -o syn -- python3 tools/synth_probe.py 1 > gpurun_out/si_probe.log 2>&1 || exit 1
grep "B=" gpurun_out/si_probe.log
python3 tools/reverse_trace.py $(find gpurun_out/si_prof -name "syn_kernel_trace.csv" | head -1) > gpurun_out/si_reverse.txt && cat gpurun_out/si_reverse.txt
for st in 3 4; do ENSVS_SMALL_STAGES=$st timeout -k 10 120 python -u tools/synth_probe.py 1 2>&1 | grep "B=" | sed "s/^/stages=$st /"; done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/si_bench.json 2> gpurun_out/si_bench.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/si_bench.json'))
s=d['synth']; r=d['roofline']
print('ms/step', round(d['ms_per_step'],2), 'gate us', round(r['launch_us'],1), 'frac', round(r['frac'],3))
print('pair acoustic ms', round(s['pair']['acoustic_ms'],1), 'rtf', round(s['pair']['rtf'],4), '6part', round(s['ensemble_6part']['rtf'],4), 'acoustic', round(s['ensemble_6part']['acoustic_ms'],1), 'voc', round(s['ensemble_6part']['vocoder_ms'],1))
"
