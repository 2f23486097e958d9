for n in 256 1024 2048; do echo "N $n" >> gpurun_out/cvar.log && PP2_N=$n PP2_REPS=50 timeout -k 10 100 python3 tools/coded_loop_timing.py >> gpurun_out/cvar.log 2>&1 || exit 1; done
