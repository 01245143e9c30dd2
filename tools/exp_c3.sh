for m in 31 3 4 8 16; do for mode in 1 3 6; do echo "mask=$m mode=$mode"; WCB_C3_MASK=$m tools/bin/wc_bench 4 c3 f64 0.999 20 3 $mode 0; done; done
