tail -2 gpurun_out/gpu_quick.log
for f in gpurun_out/bench_*.json gpurun_out/dbg_*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],4), d['config']['snapshots_in_timed'])" 2>/dev/null; done
for f in gpurun_out/dbg_c*.err; do echo $f; grep "stamps raw" $f | python -c "
import sys
for l in sys.stdin:
    v=[int(x) for x in l.split(':')[1].split()]
    print(' committer', [round(x*64/6000) for x in v[0:7]], 'checker0', [round(x*64/6000) for x in v[16:19]], 'checker1', [round(x*64/6000) for x in v[19:22]], 'drops', v[7], 'unpred', v[8]);
    print(' producers(sum over waves)', [round(x*64/6000) for x in v[24:28]], 'flagger', [round(x*64/6000) for x in v[22:24]], 'presel', [round(x*64/6000) for x in v[28:32]])"; done
