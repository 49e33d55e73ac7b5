set -o pipefail
bash tools/din_ab.sh r6b prod pf1 && bash tools/replay_grid.sh r6b 8 2x4 4x2 && bash tools/prof_fused.sh r6b_fused
