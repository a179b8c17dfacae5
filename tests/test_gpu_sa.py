"""GPU SA -> position (BWTSaValue + BWTRetrievePositionFromSAIndex)
against the compiled reference's values: every SA index of a genome with N-runs
(blocks with 'ori' offsets) and a sample of the tiny index.  Bit-exact."""
import numpy as np
import pytest

from golden_io import GOLD, INDEX
from hsa_amd import index_io

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["nrun", "tiny"])
def test_sa_position_matches_reference(name):
    from hsa_amd._lib import GpuIndex
    g = np.load(f"{GOLD}/{name}_sa.npz")
    gi = GpuIndex(*index_io.read_index(INDEX[name]))
    gi.set_sa(index_io.read_sa(INDEX[name]), index_io.read_blocks(INDEX[name]))
    got = gi.sa_positions(g["idx"])
    assert np.array_equal(got[:, 0], g["sa"])
    assert np.array_equal(got[:, 1], g["seq_id"])
    assert np.array_equal(got[:, 2], g["ori_pos"])
    assert np.array_equal(got[:, 3], g["occ_pos"])
