for f in gpurun_out/p3_c2_1.json gpurun_out/p3_c2_2.json gpurun_out/p3_c2_3.json gpurun_out/p3_c3.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), round(d['latency']['resolver_cycles_per_pod']))" 2>/dev/null; done
