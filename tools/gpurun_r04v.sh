# BASELINE configs[2] and [4] on the current tree (one setup each, after one warm-up)
set -o pipefail
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r04v
rm -rf $D; mkdir -p $D
export PYTHONPATH=$GRAFT_REPO_ROOT
PROBE_REPS=2 timeout -k 10 500 python3 -u tools/probe_configs.py sem10k aniso256 > $D/cfg.json 2> $D/cfg.err; r=$?; echo "probe rc=$r"; python3 -c "
import json
for l in open('$D/cfg.json'):
    d=json.loads(l); print(d['config'], d.get('rep'), d.get('setup_s'), d.get('rows_per_s'), d.get('ub_events'), d.get('ub_site'), d.get('ub_level'), d.get('nlevels'))"
