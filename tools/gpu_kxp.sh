mkdir -p gpurun_out/kxp
export TMPDIR=/tmp
for T in 125000 1000000; do
MJRL_AMD_LIB=mjrl_amd/lib/libmjrl_amd_prof.so timeout -k 10 200 python -u tools/kx_prof.py $T > gpurun_out/kxp/kx_prof_$T.txt 2>&1 || { echo prof failed; tail gpurun_out/kxp/kx_prof_$T.txt; exit 1; }
cat gpurun_out/kxp/kx_prof_$T.txt
done
