bash tools/ab_lib.sh a0 --steps 100 --warmup 20 && bash tools/ab_lib.sh a0 --d 1024 --dtype fp8 --reg 0.1 --steps 20 --warmup 5
