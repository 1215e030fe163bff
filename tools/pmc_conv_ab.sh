#!/bin/bash
# PMC passes (tools/pmc_conv.sh) of one conv shape on two library builds: the same counters for A and B.
# usage: tools/pmc_conv_ab.sh libA.so libB.so [conv_bench args...]   ("hip" = libnps_hip.so, "env:VAR=VAL" =
#        libnps_hip.so with that environment variable set)
A=$1; B=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
LIBDIR=neural-pde-surrogates_amd/nps_hip
for L in $A $B; do
  EV=""
  case $L in
    hip) F=$LIBDIR/libnps_hip.so ;;
    env:*) F=$LIBDIR/libnps_hip.so; EV=${L#env:} ;;
    *) F=$LIBDIR/$L ;;
  esac
  T=pmcc_$(echo ${L%.so} | tr -c 'A-Za-z0-9_\n' '_')
  env $EV NPS_HIP_LIB=$PWD/$F PMCC_TAG=$T bash tools/pmc_conv.sh "$@" || exit 1
  python3 tools/pmc_conv_summary.py gpurun_out 256 $T > gpurun_out/${T}_summary.json || exit 1
  cat gpurun_out/${T}_summary.json
done
