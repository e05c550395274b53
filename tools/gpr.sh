#!/bin/bash
# gpurun with waits on "no box / transient" outcomes (nothing charged); $1 = timeout, rest = command
T=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > ${GPR_OUT:-/tmp/gpr.out} 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off\|stopped responding while being prepared\|taken away by the GPU service\|is already running — one at a time" ${GPR_OUT:-/tmp/gpr.out} && ! grep -q "status=ok" ${GPR_OUT:-/tmp/gpr.out}; then
    echo "[gpr] transient (rc=$rc), retry $i" >&2; sleep 120; continue
  fi
  cat ${GPR_OUT:-/tmp/gpr.out}; exit $rc
done
cat ${GPR_OUT:-/tmp/gpr.out}; exit $rc
