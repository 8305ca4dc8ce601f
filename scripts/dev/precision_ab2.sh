# Developer A/B (GPU): which fast-math flag costs the parity -- the builds with
# one of -fno-associative-math / -fno-reciprocal-math / -fno-approx-func added
# to the physics unit's -ffast-math: bench step time, then the parity probes
set -u
export PYTHONUNBUFFERED=1
LIBS_AB="libtgsim.so libtgsim_assoc.so libtgsim_recip.so libtgsim_afn.so"
STEPS=1000 TASKS="ThormangWalk Gogoro" bash scripts/ab_libs.sh $LIBS_AB || exit 1
LIBS="libtgsim_assoc.so libtgsim_recip.so libtgsim_afn.so" WHICH=paper_forced,walk_forced bash scripts/dev/variant_errors.sh
