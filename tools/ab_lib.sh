#!/bin/bash
# Same-box A/B of two builds of the library: bench.py alternated A B A B (ROUNDS times), one JSON line each.
# usage: tools/ab_lib.sh TAG libA.so libB.so [bench.py args...]   (libs relative to nps_hip/, "hip" = libnps_hip.so,
#        "env:VAR=VAL" = libnps_hip.so with that environment variable set, e.g. a dev knob)
# env ROUNDS (default 2).  Output: gpurun_out/${TAG}_ab.jsonl, a summary on stdout.
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
ROUNDS=${ROUNDS:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/${TAG}_ab.jsonl
: > $O
LIBDIR=neural-pde-surrogates_amd/nps_hip
for r in $(seq 1 $ROUNDS); do
  for L in $A $B; do
    EV=""
    case $L in
      hip) F=$LIBDIR/libnps_hip.so ;;
      env:*) F=$LIBDIR/libnps_hip.so; EV=${L#env:} ;;
      *) F=$LIBDIR/$L ;;
    esac
    [ -f "$F" ] || { echo "missing $F"; exit 1; }
    env $EV NPS_HIP_LIB=$PWD/$F timeout -k 10 300 python3 bench.py --cpu-calls 0 "$@" > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_one.err \
      || { echo "bench failed on $L"; tail -20 gpurun_out/${TAG}_one.err; exit 1; }
    python3 - "$L" gpurun_out/${TAG}_one.json >> $O <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(json.dumps({"lib": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"], "frac": r.get("frac"),
                  "avg_launch_ms": r.get("avg_launch_ms"),
                  "classes": {k: v["ms"] for k, v in (r.get("conv_classes") or {}).items()}}))
EOF
    tail -1 $O
  done
done
