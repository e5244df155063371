bash s-blas_amd/tools/sessions/r04_n8knobs.sh && bash s-blas_amd/tools/sessions/r04_c5pmc.sh
