"""Prints a JSON summary {path: [dtype, shape, sum]} of every dataset of an HDF5 file (and
{group/: null} for groups) using h5py — run by tests/test_h5_cpu.py under an interpreter that has
h5py (/opt/conda/bin/python3.9 in the build container) to check that files from the in-tree
writer open in a real HDF5 library."""
import sys, json, h5py, numpy as np
out = {}
with h5py.File(sys.argv[1], "r") as f:
    def visit(name, obj):
        if isinstance(obj, h5py.Dataset):
            a = obj[()]
            out[name] = [str(a.dtype), list(np.shape(a)), float(np.asarray(a, np.float64).sum())]
        else:
            out[name + "/"] = None
    f.visititems(visit)
print(json.dumps(out))
