bash tools/ab/r06_b1split.sh > gpurun_out/r06b1split.log 2>&1 && bash tools/ab/r06_l3split.sh > gpurun_out/r06l3split3.log 2>&1
