export PYTHONPATH=$PWD/convolutional-codes_amd CCV_FANO_CAP=0
for lib in libccv_core_r02.so libccv_core_nopark.so libccv_core.so libccv_core_r02.so libccv_core_nopark.so libccv_core.so; do
  CCV_CORE_LIB=$lib timeout -k 10 200 python tools/fano_caps.py --ebn0 4 --reps 1 0 > gpurun_out/fab.txt 2>&1 || { cat gpurun_out/fab.txt; exit 1; }
  echo "$lib $(tail -1 gpurun_out/fab.txt)"
done
