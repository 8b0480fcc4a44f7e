"""The C ABI driven the way a Spark local[N] executor drives it: a C++
pthread driver (tests/abi_threads.cpp, no Python in the process) with 16
task threads calling libcyclone_blas.so's netlib symbols and libcyclone.so's
resident-dataset entry points at once; every threaded result must equal the
lone call's bits and the lone results the oracle (see the driver's header).
Reference: ml/linalg/BLAS.scala:29-30, 42-56 (one netlib instance per JVM,
shared by every task thread), docs/ml-linalg-guide.md:79-91."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "abi_threads")


def test_driver_built():
    """The driver compiles and links against the in-tree libraries and the
    oracle (__graft_entry__.build() builds it; here too when it is missing)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests")], check=True, timeout=240)
    assert os.path.exists(DRIVER)
    r = subprocess.run(["ldd", DRIVER], capture_output=True, text=True)
    assert "libcyclone_blas.so" in r.stdout and "libcyclone.so" in r.stdout
    assert "not found" not in r.stdout


@pytest.mark.gpu
def test_abi_sixteen_threads():
    r = subprocess.run([DRIVER], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    print(r.stderr[-4000:])
    assert r.returncode == 0 and r.stdout.strip().endswith("abi_threads OK"), r.stderr[-2000:]
