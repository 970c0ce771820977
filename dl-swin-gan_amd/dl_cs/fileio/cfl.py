"""BART CFL files (cfl = dl_cs/fileio/cfl.py of the reference, cfl:25-63): a text
header ``<name>.hdr`` ("# Dimensions" then the sizes, first dimension fastest)
and raw interleaved complex64 data in ``<name>.cfl``.  order='F' keeps BART's
dimension order (column-major), order='C' reverses it to numpy's row-major view
of the same bytes.  Large files are memory-mapped, not read whole."""
import numpy as np


def read_hdr(name, order='C'):
    with open(name + ".hdr") as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip() and not ln.lstrip().startswith("#")]
    dims = [int(v) for v in lines[0].split()]
    return dims[::-1] if order == 'C' else dims


def read(name, order='C', mmap=False):
    dims = read_hdr(name, order)
    n = int(np.prod(dims))
    if mmap:
        flat = np.memmap(name + ".cfl", dtype=np.complex64, mode="r", shape=(n,))
    else:
        flat = np.fromfile(name + ".cfl", dtype=np.complex64, count=n)
    return flat.reshape(dims, order=order)


def write(name, array, order='C'):
    array = np.asarray(array)
    dims = array.shape[::-1] if order == 'C' else array.shape
    with open(name + ".hdr", "w") as f:
        f.write("# Dimensions\n" + " ".join(str(int(d)) for d in dims) + " \n")
    data = array.astype(np.complex64)
    # column-major bytes: the transpose's C order is the array's Fortran order
    (data if order == 'C' else data.T).tofile(name + ".cfl")


def readcfl(name):
    return read(name, order='F')


def writecfl(name, array):
    write(name, array, order='F')
