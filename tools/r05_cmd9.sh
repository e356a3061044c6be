#!/bin/bash
# round 5: where the packed kernel's time goes (C2, timing-only variants, same box)
set -uo pipefail
R=2 AB_TAG=_r05i AB_ALLOW_WRONG=1 BENCH_ARGS="--workload c2 --steps 60" timeout -k 10 900 bash tools/ab_libs.sh base=- nomac=ablib/pk_nomac2.so noarx=ablib/pk_noarx.so nosetup=ablib/pk_nosetup.so
