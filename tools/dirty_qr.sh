#!/bin/bash
set -o pipefail
timeout -k 10 120 python -u tools/dirty_qr.py || exit 1
EIGSOL_HESS_NO_COOP=1 timeout -k 10 120 python -u tools/dirty_qr.py || exit 1
EIGSOL_QR_AED=0 timeout -k 10 120 python -u tools/dirty_qr.py || exit 1
EIGSOL_HQR_WAVE=0 timeout -k 10 120 python -u tools/dirty_qr.py || exit 1
