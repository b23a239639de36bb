# A/B: the table-only instantiation of the packed profile kernel vs the general one (C3 shape)
set -o pipefail
D=gpurun_out/${1:-r3table_kernel}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 general=netrep_amd/_lib/ab/libnotable.so table=netrep_amd/_lib/ab/libtable.so general2=netrep_amd/_lib/ab/libnotable.so table2=netrep_amd/_lib/ab/libtable.so > $D/ab_C3.txt 2>&1
