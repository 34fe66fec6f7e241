TAG=$1
tail -2 gpurun_out/c4_tests_$TAG.log
python -c "
import json; d=json.loads(open('gpurun_out/c4_$TAG.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],3), round(d['device_ms_per_step'],3), d['config']['snapshots_in_timed'], 'res', round(d['roofline']['kernel_ms_avg']*1e3,1), 'us eval', round(d['roofline']['win_eval_ms_avg']*1e3,1), 'us cyc/pod', round(d['latency']['resolver_cycles_per_pod']))"
python - <<PY
import csv,glob
for f in glob.glob('gpurun_out/prof_c4_$TAG/kt/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:60].ljust(60), r['Calls'].rjust(6), str(round(float(r['AverageNs'])/1e3,2)).rjust(8), r['Percentage'])
PY
