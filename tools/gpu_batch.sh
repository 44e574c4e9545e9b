bash tools/gpu_run.sh r05zr "pmc:FETCH_SIZE:--reg 0.1 --reg-mode full" "pmc:WRITE_SIZE:--reg 0.1 --reg-mode full"
