"""ABI equality with the reference's public headers (CPU, needs /root/reference).

Compiles a C translation unit that includes libfabric's public headers and
ours side by side and static-asserts that every enumerator, flag, error code
and mirrored struct layout is identical — so a libfabric caller's values and
structs pass straight through the drop-in boundary.
"""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/include"

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers absent")

DT = ["INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64",
      "FLOAT", "DOUBLE", "FLOAT_COMPLEX", "DOUBLE_COMPLEX", "LONG_DOUBLE",
      "LONG_DOUBLE_COMPLEX", "INT128", "UINT128", "FLOAT16", "BFLOAT16",
      "FLOAT8_E4M3", "FLOAT8_E5M2", "VOID"]
OPS = ["MIN", "MAX", "SUM", "PROD", "LOR", "LAND", "BOR", "BAND", "LXOR", "BXOR",
       "ATOMIC_READ", "ATOMIC_WRITE", "CSWAP", "CSWAP_NE", "CSWAP_LE", "CSWAP_LT",
       "CSWAP_GE", "CSWAP_GT", "MSWAP", "DIFF", "NOOP"]
COLLS = ["BARRIER", "BROADCAST", "ALLTOALL", "ALLREDUCE", "ALLGATHER",
         "REDUCE_SCATTER", "REDUCE", "SCATTER", "GATHER"]
FLAGS = ["TAGGED", "COLLECTIVE", "PEER_TRANSFER", "FETCH_ATOMIC", "COMPARE_ATOMIC"]
ERRS = ["EAGAIN", "ENOMEM", "EBUSY", "EINVAL", "ENOSYS", "EOPNOTSUPP", "EIO",
        "EOTHER", "EBADFLAGS", "ENOEQ"]


def test_abi_matches_reference_headers():
    lines = ["#include <stddef.h>", "#include <rdma/fabric.h>",
             "#include <rdma/fi_domain.h>", "#include <rdma/fi_collective.h>",
             "#include <rdma/fi_atomic.h>", "#include <rdma/fi_eq.h>",
             "#include <rdma/fi_errno.h>", '#include "lfa_fabric.h"',
             '#include "lfa_coll.h"', "#define EQ(a, b) _Static_assert((long long)(a) == (long long)(b), #a)"]
    for n in DT + OPS + COLLS + FLAGS + ERRS:
        lines.append(f"EQ(FI_{n}, LFA_{n});")
    lines += ["EQ(FI_ADDR_NOTAVAIL, LFA_ADDR_NOTAVAIL);",
              "EQ(FI_JOIN_COMPLETE, LFA_JOIN_COMPLETE);",
              "EQ(FI_ETOOSMALL, LFA_ETOOSMALL);",
              "EQ(sizeof(struct fi_atomic_attr), sizeof(struct lfa_atomic_attr));",
              "EQ(sizeof(struct fi_collective_attr), sizeof(struct lfa_collective_attr));",
              "EQ(offsetof(struct fi_collective_attr, max_members), offsetof(struct lfa_collective_attr, max_members));",
              "EQ(offsetof(struct fi_collective_attr, mode), offsetof(struct lfa_collective_attr, mode));",
              "EQ(sizeof(struct fi_cq_data_entry), sizeof(struct lfa_cq_entry));",
              "EQ(offsetof(struct fi_cq_data_entry, data), offsetof(struct lfa_cq_entry, data));",
              "EQ(sizeof(struct fi_eq_entry), sizeof(struct lfa_eq_entry));",
              "EQ(sizeof(fi_addr_t), sizeof(lfa_addr_t));",
              "int main(void) { return 0; }"]
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "abi.c")
        open(src, "w").write("\n".join(lines) + "\n")
        r = subprocess.run(["gcc", "-std=gnu11", "-I", REF, "-I",
                            os.path.join(ROOT, "include"), "-c", src, "-o",
                            os.path.join(d, "abi.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
