"""Summary-dump I/O of nlspn_eccv20_amd.replay (CPU): the reference's offset.npy /
aff.npy / gamma.npy format (src/summary/nlspnsummary.py:185-189, :265-268)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from nlspn_eccv20_amd.replay import load_dump, replay, save_dump


def _write(d, aff, gamma, off=None):
    np.save(d / "aff.npy", aff)
    np.save(d / "gamma.npy", gamma)
    if off is not None:
        np.save(d / "offset.npy", off)


def test_save_load_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    aff = rng.random((2, 9, 6, 8), dtype=np.float32)
    off = rng.standard_normal((2, 18, 6, 8)).astype(np.float32)
    off[:, 8:10] = 0.0  # reference tap K//2 = 4: planes 8, 9
    out = {"aff": torch.from_numpy(aff), "offset": torch.from_numpy(off), "gamma": torch.tensor([4.0])}
    save_dump(str(tmp_path), out)
    d = load_dump(str(tmp_path))
    assert d.kernel == (3, 3) and d.K == 8 and d.shape == (2, 6, 8)
    np.testing.assert_array_equal(d.aff, aff)
    np.testing.assert_array_equal(d.offset, off)
    np.testing.assert_array_equal(d.gamma, np.array([4.0], np.float32))


def test_no_offset_dump_from_reference_loop(tmp_path):
    """A no-offset dump: output['offset'] is None, so offset.npy is not written."""
    z = load_golden("loop_tgass_preserve")
    save_dump(str(tmp_path), {"aff": torch.from_numpy(z["aff"]), "offset": None,
                              "gamma": torch.from_numpy(z["gamma"])})
    assert not (tmp_path / "offset.npy").exists()
    d = load_dump(str(tmp_path))
    assert d.offset is None and d.kernel == (3, 3)
    np.testing.assert_array_equal(d.aff, z["aff"])


def test_kernel_inference_and_errors(tmp_path):
    aff = np.zeros((1, 17, 4, 20), np.float32)
    off = np.zeros((1, 34, 4, 20), np.float32)
    _write(tmp_path, aff, np.array([8.0], np.float32), off)
    with pytest.raises(ValueError, match="square odd kernel"):
        load_dump(str(tmp_path))
    d = load_dump(str(tmp_path), kernel=(1, 17))
    assert d.kernel == (1, 17) and d.K == 16
    with pytest.raises(ValueError, match="taps"):
        load_dump(str(tmp_path), kernel=3)


def test_rejects_bad_layouts(tmp_path):
    _write(tmp_path, np.zeros((1, 9, 4, 4), np.float32), np.array([4.0], np.float32),
           np.ones((1, 18, 4, 4), np.float32))
    with pytest.raises(ValueError, match="inserted layout"):
        load_dump(str(tmp_path))
    np.save(tmp_path / "offset.npy", np.zeros((1, 16, 4, 4), np.float32))  # raw 2K layout
    with pytest.raises(ValueError, match="inserted layout"):
        load_dump(str(tmp_path))
    np.save(tmp_path / "gamma.npy", np.array([1.0, 2.0], np.float32))
    with pytest.raises(ValueError, match="one value"):
        load_dump(str(tmp_path))


def test_missing_and_pickled_files_refused(tmp_path):
    with pytest.raises(FileNotFoundError):
        load_dump(str(tmp_path))
    np.save(tmp_path / "aff.npy", np.array([{"a": 1}], dtype=object), allow_pickle=True)
    np.save(tmp_path / "gamma.npy", np.array([4.0], np.float32))
    with pytest.raises(ValueError):  # allow_pickle=False: object arrays are never unpickled
        load_dump(str(tmp_path))


def test_replay_requires_the_hip_device(tmp_path):
    z = load_golden("loop_tgass_preserve")
    save_dump(str(tmp_path), {"aff": torch.from_numpy(z["aff"]), "offset": None,
                              "gamma": torch.from_numpy(z["gamma"])})
    with pytest.raises(RuntimeError, match="HIP"):
        replay(load_dump(str(tmp_path)), z["pred_init"], z["dep"], z["conf"], device="cpu")


def test_replay_rejects_bad_prop_time(tmp_path):
    z = load_golden("loop_tgass_preserve")
    save_dump(str(tmp_path), {"aff": torch.from_numpy(z["aff"]), "offset": None,
                              "gamma": torch.from_numpy(z["gamma"])})
    with pytest.raises(ValueError, match="prop_time"):
        replay(load_dump(str(tmp_path)), z["pred_init"], z["dep"], z["conf"], prop_time=0, device="cuda")
