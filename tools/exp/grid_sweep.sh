# grid-size A/B of the shipped schedule (tools only): workgroups = XE3_GRID,
# interleaved rounds
set -e
for round in 1 2 3 4 5 6; do
for g in ${GRIDS:-256 240}; do
  XE3_GRID=$g timeout -k 10 100 ./tools/exp/xor_exp3p 12500 5 2>/dev/null | sed "s/^{/{\"grid\": $g, \"round\": $round, /" >> gpurun_out/grid_sweep3.jsonl
done; done
