# r5g: fused sweep multiplies prod d by the chunk's product P (robust fallback per factor), unit
# exponent from sigma^2 and the model's omega^2 bound, N_HI validated: whole GPU suite + smoke, then
# c2 A/B against the previous commit (prev) over 3 rounds.
set -uo pipefail
bash tools/gpu_run.sh r5g tests smoke "ab=3=head,prev"
