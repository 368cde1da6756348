"""``alluxio runTests`` — end-to-end sanity over every ReadType x WriteType combination.

Parity: shell/src/main/java/alluxio/cli/TestRunner.java:40-200 (runs BasicOperations and
BasicNonByteBufferOperations for each combination under ``--directory``; prints
``runTest <Op> <ReadType> <WriteType>`` then ``Passed the test!``; exit code = number of failures)
and BasicOperations.java / BasicNonByteBufferOperations.java (write ints/bytes, read back, verify).
"""
from __future__ import annotations

import struct
import sys

READ_TYPES = ["CACHE_PROMOTE", "CACHE", "NO_CACHE"]
WRITE_TYPES = ["MUST_CACHE", "CACHE_THROUGH", "THROUGH", "ASYNC_THROUGH"]
OPS = ["Basic", "BasicNonByteBuffer"]


def _basic(fs, path, rt, wt) -> bool:
    """BasicOperations: write a buffer of 20 little ints, read it back through the read type."""
    n = 20
    payload = b"".join(struct.pack("<i", i) for i in range(n))
    fs.write_file(path, payload, write_type=wt)
    with fs.open_file(path, read_type=rt) as f:
        got = f.read()
    return got == payload


def _non_bytebuffer(fs, path, rt, wt) -> bool:
    """BasicNonByteBufferOperations: length-prefixed byte stream written element by element."""
    length = 20
    with fs.create_file(path, write_type=wt) as f:
        f.write(struct.pack(">i", length))
        for i in range(length):
            f.write(bytes([i & 0xFF]))
    with fs.open_file(path, read_type=rt) as f:
        got = f.read()
    if struct.unpack(">i", got[:4])[0] != length:
        return False
    return got[4:] == bytes(range(length))


def run_tests(fs, directory="/default_tests_files", operation=None, read_type=None, write_type=None,
              out=None) -> int:
    out = out or sys.stdout
    failed = 0
    for op in ([operation] if operation else OPS):
        for rt in ([read_type] if read_type else READ_TYPES):
            for wt in ([write_type] if write_type else WRITE_TYPES):
                print(f"runTest {op} {rt} {wt}", file=out)
                path = f"{directory.rstrip('/')}/{op}_{rt}_{wt}"
                try:
                    if fs.exists(path):
                        fs.delete(path)
                    ok = (_basic if op == "Basic" else _non_bytebuffer)(fs, path, rt, wt)
                except Exception as e:  # noqa: BLE001
                    print(f"Exception: {e}", file=out)
                    ok = False
                print("Passed the test!" if ok else "Failed the test!", file=out)
                failed += 0 if ok else 1
    return failed


def main(argv=None, out=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="alluxio runTests")
    ap.add_argument("--directory", default="/default_tests_files")
    ap.add_argument("--operation", default=None, choices=OPS)
    ap.add_argument("--readType", default=None, choices=READ_TYPES)
    ap.add_argument("--writeType", default=None, choices=WRITE_TYPES)
    a = ap.parse_args(argv)
    from ..client.file_system import FileSystem
    fs = FileSystem()
    try:
        return run_tests(fs, a.directory, a.operation, a.readType, a.writeType, out)
    finally:
        fs.close()
