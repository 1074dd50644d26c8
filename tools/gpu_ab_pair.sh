cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for round in 1 2 3; do
for t in pre default; do
  if [ $t = default ]; then L=sonido-sonar_amd/lib/libsonar_gpu.so; else L=sonido-sonar_amd/lib_$t/libsonar_gpu.so; fi
  SONAR_LIB=$PWD/$L ITERS=30 timeout -k 10 200 python3 tools/fp_microbench.py mfcc mfcc_f64p mfcc > gpurun_out/ab.jsonl 2>gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  sed "s/^/$t /" gpurun_out/ab.jsonl | tee -a gpurun_out/r06ar_ab.log
done
done
