"""The demapper's exact shortcuts against the forms they replace (DESIGN.md §3,
k_demap_planes): the f32 square root on [1, 2] (raw v_sqrt_f32 plus the
compiler's +-1 ulp correction) for EVERY f32 in [1, 2] against sqrtf and the
correctly rounded square root, and the finite-input |z| against numpy's |z|
restated with its inf / NaN rules (npm::cabs_np, the form the oracle-pinned
demap tests already cover) on 2^26 random finite pairs in f32 and f64; the f64 division and square root
without their range scaling (TDEC_DM_FAST64) against the compiler's sequences on
2^28 random operands of the demapper's ranges.
Bit-identical, or the fast path would not be the full scan's result."""
import ctypes as C

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from modulations_amd import _native  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("which,n", [(0, 0), (1, 1 << 26), (2, 1 << 26), (4, 1 << 28)],
                         ids=["sqrt_1_2_exhaustive", "cabs_f32", "cabs_f64", "unscaled_f64_div_sqrt"])
def test_demap_shortcuts_bit_identical(which, n):
    bad = C.c_longlong(-1)
    _native.check(_native.lib().tdec_selftest(0, which, n, 0x5EED0000 + which, C.byref(bad)))
    assert bad.value == 0
