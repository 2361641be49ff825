# config-2 tally time vs chunk size (wave-tiles per chunk), direct commits only (FR_LOG=0)
mkdir -p gpurun_out
out=gpurun_out/r03_chunk.log; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 5 120 python -u scripts/diag_scale.py 100000000 3700 >> $out 2>&1 || { echo "FAILED $*" >> $out; exit 1; }; }
for c in 320 448 640 896 1280; do run FR_LOG=0 FR_CHUNK_TILES=$c; done
grep -v amdgpu.ids $out | sed -e 's/ lines=.*U=/ U=/' -e "s/'spin_max.*//"
