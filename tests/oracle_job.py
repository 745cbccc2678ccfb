"""Background oracle jobs for tests/test_gpu_fullsize_oracle.py: the C oracle's
whole proofs of seeded NCOLS x NCOLS permutation traces, one after another,
each written to its OUT file (atomically: the reader sees a whole proof or
nothing).  conftest.py starts this when the tests are selected, so the
oracle's minutes of host work overlap the rest of the GPU suite instead of
adding to it.
Usage: python tests/oracle_job.py THREADS OUT:LOG_N:NCOLS [OUT:LOG_N:NCOLS ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import cref  # noqa: E402


def main():
    threads = int(sys.argv[1])
    p = cref.setup()
    for job in sys.argv[2:]:
        out, log_n, ncols = job.rsplit(":", 2)
        log_n, ncols = int(log_n), int(ncols)
        tb, w = cref.gen_perm_trace(p, log_n, ncols)
        proof = cref.prove(p, tb, 1 << log_n, w, cref.perm_air(ncols), nthreads=threads)
        del tb
        tmp = out + ".part"
        with open(tmp, "wb") as f:
            f.write(proof)
        os.replace(tmp, out)


if __name__ == "__main__":
    main()
