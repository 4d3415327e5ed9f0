cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out; OUT=gpurun_out/chunk_ab.jsonl; : > $OUT
L=cuda-bezier-triangle-raytracer_amd/lib
for r in 1 2; do
 for spec in "base 2" "chunk22 2" "chunk22 4" "chunk24 2"; do
  set -- $spec
  if [ $1 = base ]; then lib=$L/libbzr.so; else lib=$L/$1/libbzr.so; fi
  BZR_LIBRARY=$PWD/$lib timeout -k 10 240 python bench.py --config cfg5 --pipeline staged --inflight $2 --cpu-baseline off > gpurun_out/chunk_one.log 2>&1 || exit $?
  grep '^{' gpurun_out/chunk_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant':'$1','inflight':$2,'rep':$r,'mrays_s':d['value'],'ms_per_step':d['ms_per_step']}))" | tee -a $OUT
 done
done
