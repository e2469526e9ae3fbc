# round 3 profiles: stateless configs (kernel stats, traffic, TCC, SQ) then the stateful rows (F1, D1)
set -o pipefail
bash tools/profile_round.sh r3 "C1 C2 C3 C4" && bash tools/profile_stateful.sh r3
