set -u
export TMPDIR=/tmp
OUT=gpurun_out/p1d
mkdir -p $OUT
for v in 1d_base 1d_noreg; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum"; do
    i=$((i+1))
    CUZFP_HIP_LIB=$PWD/build/xvar/$v/libcuzfp_hip.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/$v/g$i -o run -- python tools/kernel_probe.py --dims 1 --size 1048576 > $OUT/${v}_g$i.log 2>&1
    echo "$v g$i exit $?"
  done
  python tools/counters.py $OUT/$v
done
