for s in 3 4 5 6 7; do timeout -k 5 60 tools/micro/gpubin/dx_diag_0 $s 1 || exit 1; done
