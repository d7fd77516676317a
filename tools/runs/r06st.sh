bash tools/runs/r06s.sh > gpurun_out/r06s.txt 2>&1; tail -60 gpurun_out/r06s.txt; bash tools/runs/r06t.sh
