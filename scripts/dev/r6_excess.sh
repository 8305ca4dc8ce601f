# Developer study (GPU): scripts/dev/r6_gogoro_excess.py under each library in
# LIBS (thormang_isaacgym_amd/<lib>), one process per library
set -u
mkdir -p gpurun_out/excess
export PYTHONUNBUFFERED=1
for l in ${LIBS:-libtgsim.so}; do
  TG_LIB_PATH=thormang_isaacgym_amd/$l timeout -k 10 300 python -u scripts/dev/r6_gogoro_excess.py ${ARGS:-} > gpurun_out/excess/$l.log 2>&1 || { tail -5 gpurun_out/excess/$l.log; exit 1; }
  grep -v '^==' gpurun_out/excess/$l.log | grep -v Warn
done
