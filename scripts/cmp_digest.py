#!/usr/bin/env python3
"""Compare two state_digest.py outputs: number of differing entries and the largest difference."""
import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    d = np.abs(a[k] - b[k])
    print(f"{k}: {int((a[k] != b[k]).sum())} of {a[k].size} differ, max |diff| {d.max():.3e}")
