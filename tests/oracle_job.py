"""Background oracle job for tests/test_gpu_fullsize_oracle.py: the C oracle's
whole proof of the seeded 3x3 permutation trace at 2^LOG_N rows, written to
OUT.  conftest.py starts it when the test is selected, so its ~5 minutes of
host work overlap the rest of the GPU suite instead of adding to it.
Usage: python tests/oracle_job.py LOG_N THREADS OUT"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import cref  # noqa: E402


def main():
    log_n, threads, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    p = cref.setup()
    tb, w = cref.gen_perm_trace(p, log_n, 3)
    proof = cref.prove(p, tb, 1 << log_n, w, cref.perm_air(3), nthreads=threads)
    tmp = out + ".part"
    with open(tmp, "wb") as f:
        f.write(proof)
    os.replace(tmp, out)  # the reader sees the whole proof or nothing


if __name__ == "__main__":
    main()
