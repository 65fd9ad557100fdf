mkdir -p gpurun_out/st2
for v in tile; do
GSR_RENDER=$v GSR_LIBRARY=$PWD/gaussian_splatting_amd/lib/libgsr_stamps.so timeout -k 10 300 python tools/stamps.py > gpurun_out/st2/stamps_$v.json 2>&1 || exit 1
done
