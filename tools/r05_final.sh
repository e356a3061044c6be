#!/bin/bash
# round 5 final build: profiles (kernel traces + PMC passes, C1 and C2), then
# the round check (GPU suite, smoke, bench lines, record path, loopbacks)
set -uo pipefail
timeout -k 10 1000 bash tools/profile_round.sh r05v || exit 1
timeout -k 10 1000 bash tools/profile_round.sh r05v_c2 --workload c2 || exit 1
timeout -k 10 1100 bash tools/round_check.sh r05vc
