set -e
cd scripts/lab
for s in "fwd ffn1" "dgrad ffn1" "wgrad ffn1 s7" "fwd qkv"; do
  timeout -k 10 120 ./gemm_lab 20 "$s" "256x128 4x2 bk32"
  timeout -k 10 120 ./gemm_lab_nosplit 20 "$s" "256x128 4x2 bk32"
done
