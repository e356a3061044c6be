#!/bin/bash
# round 5 final build (header docs): profiles (kernel traces + PMC passes, C1
# and C2); the round check runs after their traffic summary is committed
set -uo pipefail
timeout -k 10 1000 bash tools/profile_round.sh r05u || exit 1
timeout -k 10 1000 bash tools/profile_round.sh r05u_c2 --workload c2 || exit 1
