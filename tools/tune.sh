set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tunableop
TB_TUNABLEOP_DIR=gpurun_out/tunableop timeout -k 10 1000 python bench.py --steps 1 --warmup 1 --tune-gemms > gpurun_out/tune.log 2>&1
echo TUNED; ls -la gpurun_out/tunableop; wc -l gpurun_out/tunableop/*.csv
TB_TUNABLEOP_DIR=gpurun_out/tunableop timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/tuned_bench.log 2>&1
tail -1 gpurun_out/tuned_bench.log | cut -c1-200
