set -e
cd scripts/lab
export LAB_PASSES=3
for s in "fwd ffn1" "dgrad ffn1" "wgrad ffn1 s7" "fwd qkv" "fwd ffn2" "fwd out" "dgrad ffn2" "wgrad qkv s9" "wgrad ffn2 s5" "co pv"; do
  timeout -k 10 150 ./gemm_lab 20 "$s" "x6"
done
