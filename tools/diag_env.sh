set -o pipefail
cd /root/repo
C="m224b2 m224 m64"
DIAG_TAG=default timeout -k 10 200 python tools/diag_numerics2.py $C
DIAG_TAG=nowino MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_FFT=0 timeout -k 10 200 python tools/diag_numerics2.py $C
DIAG_TAG=direct MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_FFT=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 timeout -k 10 200 python tools/diag_numerics2.py $C
DIAG_TAG=gemm MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_FFT=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 MIOPEN_DEBUG_CONV_DIRECT=0 timeout -k 10 200 python tools/diag_numerics2.py $C
