# iteration on the GPU box: focused parity (plain resolver, fuzz, extensions, server), then bench lines
# usage: tools/gpu_iter3.sh <tag> [workload...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "not full_size and not config5_full and not faithful" tests/test_gpu_fuzz.py \
  tests/test_gpu_extensions.py tests/test_gpu_serve.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for w in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w > gpurun_out/${TAG}_${w}.json 2> gpurun_out/${TAG}_${w}.err || exit 1
  python - "$TAG" "$w" <<'PY'
import json,sys
t,w=sys.argv[1:]
d=json.loads(open(f"gpurun_out/{t}_{w}.json").read().strip().splitlines()[-1])
L=d["latency"]
st=L.get("stages",{}); print(w, round(d["value"]), round(L["resolver_cycles_per_pod"]), round(d["ms_per_step"],3), json.dumps(st.get("committer")))
PY
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-stages --extensions --ext-filters-only > gpurun_out/${TAG}_c2_extf.json 2> gpurun_out/${TAG}_c2_extf.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/${TAG}_c2_extf.json').read().strip().splitlines()[-1]);print('c2_extf', round(d['value']), round(d['latency']['resolver_cycles_per_pod']))"
