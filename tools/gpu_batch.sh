bash tools/ab_lib.sh g2 --steps 100 --warmup 20 && bash tools/ab_lib.sh e1 --steps 100 --warmup 20
