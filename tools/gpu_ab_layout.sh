# A/B of context / hardware-queue layouts on C2: each LAYOUTS entry "ENV;ARGS" (ENV "-" = none, ARGS with
# '+' for spaces) runs the bench once: gpurun_out/layout_<i>.json
set -u
cd "$GRAFT_REPO_ROOT"
i=0
for e in $LAYOUTS; do
  i=$((i+1))
  envs=${e%%;*}; args=${e#*;}
  envs=$( [ "$envs" = "-" ] && echo "" || echo "$envs" | tr ',' ' ')
  args=$(echo "$args" | tr '+' ' ')
  env $envs timeout -k 10 300 python bench.py --no-cpu --h2d off $args > gpurun_out/layout_$i.json 2> gpurun_out/layout_$i.err
  rc=$?; case $rc in 0) ;; *) echo "layout[$i] rc=$rc"; exit $rc;; esac
  python3 -c "import json;l=[x for x in open('gpurun_out/layout_$i.json') if x.startswith('{')][-1];print('$i', '$e', json.loads(l)['value'])"
done
