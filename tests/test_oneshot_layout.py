"""The one-shot kernel's slot layout is checked on the host before any launch
(lfa_kernels.hpp launch_oneshot): both epoch parities live in FIXED halves of
SYM_IN, parity_off apart, and a layout whose n slots do not fit below
parity_off is refused.  Round 3's mixed in-flight failure came from parity
bases that moved with each operation's slot size; these
tests pin the argument rules without a GPU (every case returns before the
first HIP call)."""
import ctypes

import pytest

from libfabric_amd import coll
from libfabric_amd.atomic import LFA_EINVAL

FI_SUM, FI_FLOAT = 2, 8
BASE = 1 << 30                       # never dereferenced: every case is refused


def _args(n=4, count=1024, slot=4096, parity_off=1 << 20, sym_align=0):
    sym = (ctypes.c_void_p * n)(*[BASE + k * (4 << 20) + sym_align for k in range(n)])
    a = coll.OneShot(BASE - (1 << 20), BASE - (2 << 20), count, -1,
                     ctypes.cast(sym, ctypes.c_void_p), slot, parity_off, 2 << 20, n, 0, 1,
                     BASE - (3 << 20), 1, 1000)
    return a, sym


@pytest.mark.parametrize("kw", [
    dict(parity_off=3 * 4096),                 # 4 slots of 4 KiB do not fit below it
    dict(parity_off=0),
    dict(parity_off=(1 << 20) + 16),           # not a multiple of 256
    dict(slot=4096 + 16),                      # slot not a multiple of 256
    dict(slot=2048),                           # smaller than the 4 KiB part
    dict(sym_align=16),                        # workspace not 256-B aligned
])
def test_layout_refused(kw):
    a, _sym = _args(**kw)
    with pytest.raises(coll.CollError) as e:
        coll.oneshot_reduce(FI_SUM, FI_FLOAT, a, None)
    assert e.value.rc == -LFA_EINVAL


def test_struct_matches_header():
    """ctypes mirror of struct lfa_oneshot: parity_off right after
    slot_bytes (lfa_signal.h)."""
    f = [name for name, _ in coll.OneShot._fields_]
    assert f.index("parity_off") == f.index("slot_bytes") + 1
    assert coll.OneShot.parity_off.offset == coll.OneShot.slot_bytes.offset + 8
