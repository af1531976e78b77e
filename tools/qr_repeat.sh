#!/bin/bash
set -o pipefail
timeout -k 10 150 python -u tools/qr_repeat.py 60 || exit 1
EIGSOL_HESS_NO_COOP=1 timeout -k 10 150 python -u tools/qr_repeat.py 60 || exit 1
EIGSOL_QR_AED=0 timeout -k 10 150 python -u tools/qr_repeat.py 60 || exit 1
EIGSOL_QR_GROUPS=1 timeout -k 10 150 python -u tools/qr_repeat.py 60 || exit 1
