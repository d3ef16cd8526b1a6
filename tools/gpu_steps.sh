#!/bin/bash
# One parametrised GPU-box runner (round 5; replaces the per-experiment
# tools/gpu_r4*.sh one-offs).  Run from the repo root on the box:
#   gpurun -- 'bash tools/gpu_steps.sh TAG STEP [STEP ...]'
# Steps run in order, each under its own `timeout -k`; the first failure ends
# the call (no GPU step runs after a fault, abort or timeout).  Outputs go to
# gpurun_out/TAG/NN_<kind>.{log,json}.  A step is KIND=ARGS with ARGS passed
# word-split to the tool (use ',' for spaces inside one step):
#   test=<pytest args>      python -u -m pytest -x -v --timeout 300 --timeout-method thread <args>
#   bench=<bench.py args>   python -u bench.py <args>          -> NN_bench.json (the JSON line)
#   prof=<bench.py args>    rocprofv3 --kernel-trace --stats of bench.py <args> -> NN_prof/
#   py=<script args>        python -u <script> <args>
#   pmc=<checkpoint tag>    HBM traffic of the headline launch (tools/pmc_traffic.sh: one rocprofv3
#                           --pmc pass per counter) -> NN_pmc/pmc_traffic.json; the following
#                           bench steps read it (--traffic-json) unless they pass their own
#   sh=<script args>        bash <script> <args> (e.g. tools/gpu_strong_split_c5.sh TAG)
#   env=K=V                 export K=V for the following steps
#   budget=SECONDS          timeout of the following steps (default 600)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
T=600
n=0
for step in "$@"; do
  kind=${step%%=*}
  args=${step#*=}
  args=${args//,/ }
  n=$((n + 1))
  p=$(printf "%s/%02d_%s" "$O" "$n" "$kind")
  case $kind in
    env) export "${step#env=}"; echo "env ${step#env=}"; continue ;;
    budget) T=$args; continue ;;
    test) timeout -k 10 "$T" python -u -m pytest -x -v --timeout 300 --timeout-method thread $args > "$p.log" 2>&1 ;;
    bench) timeout -k 10 "$T" python -u bench.py ${ZS_TRAFFIC_JSON:+--traffic-json $ZS_TRAFFIC_JSON} $args > "$p.json" 2> "$p.err" ;;
    prof) (cd /tmp && timeout -k 10 "$T" rocprofv3 --kernel-trace --stats -d "$p" -o run -- python3 "$R/bench.py" $args > "$p.json" 2> "$p.err") ;;
    py) timeout -k 10 "$T" python -u $args > "$p.log" 2>&1 ;;
    sh) timeout -k 10 "$T" bash $args > "$p.log" 2>&1 ;;
    pmc) PMC_OUT="$p" PMC_TAG="$args" bash tools/pmc_traffic.sh > "$p.log" 2>&1 && [ -s "$p/pmc_traffic.json" ] &&
         export ZS_TRAFFIC_JSON="$p/pmc_traffic.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $n $kind rc=$rc"
  case $kind in
    test) grep -E "passed|failed|FAILED|Error" "$p.log" | tail -4 ;;
    bench|prof) python3 -c "
import json,sys
d=json.loads(open('$p.json').read().strip().splitlines()[-1])
print('value',d.get('value'),'ms',d.get('ms_per_step'),'exact',d.get('verified_bit_exact'),d.get('path_stats'))
print('stages',d.get('roofline',{}).get('stages_ms_avg'))" 2>&1 | tail -3 ;;
    py|sh) tail -5 "$p.log" ;;
    pmc) python3 -c "import json;d=json.load(open('$p/pmc_traffic.json'));print('traffic',d['hbm_bytes_per_launch'],d.get('source_sha256'))" ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done
