#!/bin/bash
# Effective shader clock probe: GRBM_GUI_ACTIVE / GRBM_COUNT / SQ_BUSY_CYCLES per dispatch with the kernel trace (C2, C3).
cd /tmp && for wl in c2_s1024 c3_s1024_reflect; do timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/clk_$wl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-anchor --no-cold > $GRAFT_REPO_ROOT/gpurun_out/clk_$wl.log 2>&1 || exit 1; done
