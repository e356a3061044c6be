#!/bin/bash
# round 5 final build (three-slot record pipeline): kernel-trace + PMC passes
# for C1 and C2 (tools/profile_round.sh)
set -uo pipefail
timeout -k 10 1000 bash tools/profile_round.sh r05z || exit 1
timeout -k 10 1000 bash tools/profile_round.sh r05z_c2 --workload c2 || exit 1
