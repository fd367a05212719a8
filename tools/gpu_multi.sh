#!/bin/bash
# Several measurement steps in one GPU call, each under its own time limit,
# stopping at the first failure.  Steps are given as arguments:
#   test:<pytest -k expr>   proj:<shapes>|<variants>   emu:<workload>|<ranks>|<variants>
#   bench:<bench.py args>   edge:<workload>|<variants>
# usage: bash tools/gpu_multi.sh <tag> <step> [<step> ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
i=0
for STEP in "$@"; do
  i=$((i+1))
  KIND=${STEP%%:*}; ARG=${STEP#*:}
  OUT=gpurun_out/${TAG}_${i}_${KIND}
  echo "== step $i: $KIND $ARG"
  case $KIND in
    test)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests -k "$ARG" > $OUT.log 2>&1 || { echo "FAILED"; tail -40 $OUT.log; exit 1; }
      tail -1 $OUT.log ;;
    proj)
      S=${ARG%%|*}; V=${ARG#*|}
      timeout -k 10 600 python3 -u tools/proj_bench.py --shapes "$S" --variants "$V" --out $OUT.json > $OUT.log 2>&1 || { echo "FAILED"; tail -20 $OUT.log; exit 1; }
      grep '^{' $OUT.log ;;
    emu)
      W=${ARG%%|*}; REST=${ARG#*|}; R=${REST%%|*}; V=${REST#*|}
      timeout -k 10 900 python3 -u tools/emu_probe.py --workload $W --ranks $R --variants "$V" > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    bench)
      timeout -k 10 900 python3 -u bench.py $ARG --detail-out $OUT.detail.json > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    edge)
      W=${ARG%%|*}; V=${ARG#*|}
      timeout -k 10 600 python3 -u tools/edge_ab.py --workload $W --variants "$V" > $OUT.json 2> $OUT.err || { echo "FAILED"; tail -20 $OUT.err; exit 1; }
      cat $OUT.json ;;
    *) echo "unknown step $KIND"; exit 2 ;;
  esac
done
echo "ALL OK"
