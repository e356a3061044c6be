#!/bin/bash
# round 5: energy per record of the product and the C1 timing-only variants (same box)
set -uo pipefail
R=2 AB_TAG=_r05c AB_ALLOW_WRONG=1 timeout -k 10 900 bash tools/ab_libs.sh base=- nomac=ablib/wpr_nomac.so nomfma=ablib/wpr_nomfma.so noff=ablib/wpr_noff.so noepi=ablib/wpr_noepi.so nopro=ablib/wpr_nopro.so
