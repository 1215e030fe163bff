# 1x1 DMA-stream kernel: parity (conv_bench --check vs torch CPU) and A/B against the register-staged kernels
export TMPDIR=/tmp
SHAPES=("--cin 388 --cout 192 --hw 260" "--cin 196 --cout 192 --hw 256" "--cin 84 --cout 192 --hw 256"
        "--cin 192 --cout 192 --hw 132" "--cin 20 --cout 75 --hw 64" "--cin 48 --cout 128 --hw 40")
for D in 1 0; do
  for A in "${SHAPES[@]}"; do
    echo "dma=$D $A"
    NPS_X1_DMA=$D timeout -k 10 120 python -u tools/conv_bench.py --prec x3f16 --b 16 --k 1 --gn 0 $A --check 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
