# Developer A/B (GPU): bench step time of the default library against the
# precise-math builds, then the parity probes nearest the bar under the two
# partial builds (scripts/dev/variant_errors.py)
set -u
export PYTHONUNBUFFERED=1
STEPS=1000 TASKS="ThormangWalk Gogoro" bash scripts/ab_libs.sh libtgsim.so libtgsim_precise.so libtgsim_sincos.so libtgsim_nofast.so libtgsim.so || exit 1
LIBS="libtgsim_sincos.so libtgsim_nofast.so" WHICH=paper_forced,walk_forced bash scripts/dev/variant_errors.sh
