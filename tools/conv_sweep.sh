#!/bin/bash
# representative U-FNO C3 (B=16) conv shapes; each line one launch shape
set -e
P="python tools/conv_bench.py"
$P --cin 388 --cout 192 --k 3 --hw 260 --b 16 --gn 1 --check
$P --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 1
$P --cin 196 --cout 192 --k 3 --hw 256 --b 16 --gn 1
$P --cin 388 --cout 192 --k 1 --hw 260 --b 16 --gn 0
$P --cin 196 --cout 192 --k 3 --hw 127 --b 16 --gn 1
$P --cin 128 --cout 128 --k 5 --dil 4 --circ 8 --hw 256 --b 16 --gn 0 --check
