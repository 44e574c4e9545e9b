bash tools/ab_lib.sh z0 --reg 0.1 --reg-mode full --steps 10 --warmup 3
