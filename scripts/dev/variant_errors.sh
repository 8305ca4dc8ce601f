# Developer probe (GPU): scripts/dev/variant_errors.py under each library named
# in LIBS (thormang_isaacgym_amd/<lib>), one process per library
set -u
mkdir -p gpurun_out/variants
export PYTHONUNBUFFERED=1
for l in ${LIBS:-libtgsim.so}; do
  TG_LIB_PATH=thormang_isaacgym_amd/$l timeout -k 10 900 python -u scripts/dev/variant_errors.py ${WHICH:-paper_forced,walk_forced,walk_dr,walk_stand} ${SOLVER:-} > gpurun_out/variants/$l.log 2>&1 || { tail -5 gpurun_out/variants/$l.log; exit 1; }
  grep "solver=" gpurun_out/variants/$l.log
done
