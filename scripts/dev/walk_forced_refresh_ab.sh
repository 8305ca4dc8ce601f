# Developer A/B (GPU): the 8192-env teacher-forced walk with the fp32 control, the
# default library under TGS and PGS, then the TG_PGS_REFRESH build under TGS
set -u
mkdir -p gpurun_out/s4
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u scripts/dev/r4_walk_forced.py 1,0 > gpurun_out/s4/forced_default.log 2>&1 || { tail -5 gpurun_out/s4/forced_default.log; exit 1; }
cat gpurun_out/s4/forced_default.log | grep solver_type | cut -c1-400
TG_LIB_PATH=thormang_isaacgym_amd/libtgsim_refresh.so timeout -k 10 600 python -u scripts/dev/r4_walk_forced.py 1 > gpurun_out/s4/forced_refresh.log 2>&1 || { tail -5 gpurun_out/s4/forced_refresh.log; exit 1; }
cat gpurun_out/s4/forced_refresh.log | grep solver_type | cut -c1-400
