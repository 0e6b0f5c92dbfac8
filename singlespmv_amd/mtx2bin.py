"""Matrix Market -> SPMVCSR1 binary cache.

    python -m singlespmv_amd.mtx2bin in.mtx out.csrbin [--csr5] [--no-expand]

Default semantics are the reference's LoadSparseMatrix (src/util.cpp:30-66:
banner ignored, rows column-sorted); --csr5 uses the CSR5 benchmark's
banner-aware loader (CSR5_cuda/main.cu:157-306: pattern/integer fields,
symmetric expansion).  Later runs load the cache with load_csr_bin in a
fraction of the parse time.
"""
import argparse
import sys
import time

import singlespmv_amd as sp


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("mtx")
    ap.add_argument("out")
    ap.add_argument("--csr5", action="store_true", help="banner-aware CSR5 loader semantics")
    ap.add_argument("--no-expand", action="store_true", help="with --csr5: keep symmetric files as stored")
    a = ap.parse_args(argv)
    t0 = time.time()
    if a.csr5:
        m, n, rp, col, val, info = sp.load_mtx_csr(a.mtx, sort_columns=False, expand=not a.no_expand)
    else:
        A = sp.load_sparse_matrix(a.mtx)
        m, n, col, val = A.nRow, A.nCol, A.col_idx, A.val
        rp = sp.coo_to_csr(m, A.row_idx)
        info = {}
    t1 = time.time()
    sp.save_csr_bin(a.out, m, n, rp, col, val)
    print(f"{a.mtx}: {m} x {n}, {len(val)} nnz {info} parsed in {t1 - t0:.2f} s, "
          f"wrote {a.out} in {time.time() - t1:.2f} s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
