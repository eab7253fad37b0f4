set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -2 $O/t.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
cat $O/b.json
timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-extra --size-mib 64 --steps 50 > $O/b64.json 2>> $O/b.err && cat $O/b64.json
