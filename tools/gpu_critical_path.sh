set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/${1:-critpath}
mkdir -p $out
DEBUG_WRITE_AUDITLOG=$PWD/$out/a1.jsonl timeout -k 10 200 python bench.py --steps 200 --burst 0 --probe-sample 0 --no-configs > $out/bench_n1_audit.log 2>&1 || exit 1
python tools/critical_path.py $out/a1.jsonl --namespace-prefix bench- --name-prefix nb-s > $out/critical_path_n1.json || exit 1
DEBUG_WRITE_AUDITLOG=$PWD/$out/a4.jsonl timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29934 bench.py --gpus 4 --steps 100 --warmup 5 --burst 0 --probe-sample 0 --no-configs > $out/bench_n4_audit.log 2>&1 || exit 1
python tools/critical_path.py $out/a4.jsonl --namespace-prefix bench- --name-prefix nb-s > $out/critical_path_n4.json || exit 1
rm -f $out/a1.jsonl $out/a4.jsonl
echo done
