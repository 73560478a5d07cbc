# Kernel trace of a bench.py step on one MI355X: per-kernel table (rocpd_summary.py) and idle gaps
# (rocpd_timeline.py) into gpurun_out/<tag>/. Usage (through gpurun, from the repo root):
#   bash tools/profile_step.sh <tag> [bench.py args...]      e.g. bash tools/profile_step.sh prof_r50
set -o pipefail
R=$(pwd)
TAG=${1:-prof}; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
D=/tmp/tfk_prof_$TAG; rm -rf $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace -d $D -o rn -- python3 $R/bench.py --steps 10 --warmup 3 "$@" > $O/bench.log 2>&1 || exit 3
DB=$(find $D -name "*.db" | head -1)
python3 $R/tools/rocpd_summary.py $DB --steps 13 > $O/kernels.txt 2>&1
# step windows aligned on the model's first kernel
case "$*" in *bert*|*transformer*) FIRST=embed_fwd ;; *) FIRST=stem_fwd ;; esac
python3 $R/tools/rocpd_timeline.py $DB --steps 13 --last 3 --top 30 --first $FIRST > $O/timeline.txt 2>&1
