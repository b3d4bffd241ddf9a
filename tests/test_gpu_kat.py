"""The reference's known-answer tests, run on the GPU product path."""
import pytest

import kat_cases

pytestmark = pytest.mark.gpu

GPU_KATS = [k for k in kat_cases.ALL_KATS]


@pytest.mark.parametrize("kat", GPU_KATS, ids=lambda f: f.__name__)
def test_gpu_kat(product, kat):
    kat(product)


def test_gpu_path_a_in_path_b(product):
    l1 = ("1", "1/2", "2", "2/1")
    l2 = ("2", "2/3", "3", "3/2")
    f = product.pathAInPathB
    assert f([l1], [l1, l2]) and not f([l2, l1], [l1, l2])
