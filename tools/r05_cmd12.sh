#!/bin/bash
# round 5: the 16 KiB kernel at one workgroup per CU (the residency two blocks per lane would need), same box
set -uo pipefail
R=3 AB_TAG=_r05j timeout -k 10 900 bash tools/ab_libs.sh base=- one_wg=ablib/wpr_1wg.so
