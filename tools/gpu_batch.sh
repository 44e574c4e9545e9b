bash tools/ab_lib.sh c0 --reg 0.1 --reg-mode full --steps 10 --warmup 3 && bash tools/ab_lib.sh c1 --reg 0.1 --reg-mode full --steps 10 --warmup 3
