cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/tw
timeout -k 10 400 python scripts/ab.py --config cfg4 --pipeline fused --rounds 3 base tw7 tw8 > gpurun_out/tw/cfg4.jsonl 2> gpurun_out/tw/cfg4.err || exit $?
timeout -k 10 300 python scripts/ab.py --config cfg2 --pipeline fused --rounds 3 base tw7 tw8 > gpurun_out/tw/cfg2.jsonl 2> gpurun_out/tw/cfg2.err || exit $?
L=cuda-bezier-triangle-raytracer_amd/lib
: > gpurun_out/tw/bench.jsonl
for r in 1 2; do for v in base tw7 tw8; do
  if [ $v = base ]; then lib=$L/libbzr.so; else lib=$L/$v/libbzr.so; fi
  BZR_LIBRARY=$PWD/$lib timeout -k 10 240 python bench.py --cpu-baseline off > gpurun_out/tw/one.log 2>&1 || exit $?
  grep '^{' gpurun_out/tw/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant':'$v','rep':$r,'mrays_s':d['value'],'ms_per_step':d['ms_per_step'],'verified':d['config']['frame_verified']['oracle_digests']['ok']}))" >> gpurun_out/tw/bench.jsonl
done; done
