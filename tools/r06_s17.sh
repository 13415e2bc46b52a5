# round-6 session 17: every BASELINE config line on the final default (tools/bench_configs.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/session.sh r06s17 configs
