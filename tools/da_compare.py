"""Compare two tools/da_dump.py outputs bit for bit.  usage: da_compare.py A.npz B.npz"""
import sys

import numpy as np

A, B = np.load(sys.argv[1]), np.load(sys.argv[2])
bad = 0
for k in A.files:
    same = np.array_equal(A[k], B[k])
    bad += not same
    print(f"{k:14s} {'identical' if same else 'DIFFERENT max %.3e' % np.max(np.abs(A[k] - B[k]))}")
sys.exit(1 if bad else 0)
