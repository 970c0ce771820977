for v in BASE NODBIAS NODQ NOSTAGE NODBIASDABL_NODQ; do echo "== $v"; DLCS_HIP_LIB=$PWD/abl_tmp/lib_$v.so timeout -k 10 60 python tools/attn_bench.py 10 || exit 1; done
