"""radler.WorkTable / WorkTableEntry bindings, restated from the reference's
python/test/test_work_table.py (cpp/work_table.cc behaviour)."""
import numpy as np
import pytest

from radler_import import radler as rd


def test_work_table_entry():
    e = rd.WorkTableEntry()
    assert e.image_weight == 0.0 and e.central_frequency == 0.0
    assert e.band_start_frequency == 0.0 and e.band_end_frequency == 0.0
    assert e.original_channel_index == 0 and e.original_interval_index == 0
    assert e.mask_channel_index == 0
    e.image_weight = 1.25
    e.band_start_frequency, e.band_end_frequency = 50.0e6, 60.0e6
    e.original_channel_index, e.original_interval_index = 2, 1
    e.mask_channel_index = 42
    assert e.central_frequency == (50.0e6 + 60.0e6) / 2.0
    assert (e.original_channel_index, e.original_interval_index, e.mask_channel_index) == (2, 1, 42)


def test_zero_groups():
    t = rd.WorkTable([], 0, 0)
    assert t.original_groups == [[]]
    assert t.deconvolution_groups == [[0]]


@pytest.mark.parametrize("n_orig,n_deconv", [(-2, 1), (10, -1)])
def test_negative_groups(n_orig, n_deconv):
    with pytest.raises(TypeError):
        rd.WorkTable([], n_orig, n_deconv)


@pytest.mark.parametrize("n_orig,n_deconv", [(4, 12), (12, 4)])
def test_multiple_deconvolution_groups(n_orig, n_deconv):
    t = rd.WorkTable([], n_orig, n_deconv)
    assert len(t.original_groups) == n_orig
    assert not any(t.original_groups)
    assert len(t.deconvolution_groups) == min(n_deconv, n_orig)
    n_sub = n_orig // min(n_orig, n_deconv)
    for i, sub in enumerate(t.deconvolution_groups):
        assert sub == list(range(i * n_sub, (i + 1) * n_sub))


@pytest.mark.parametrize("offset", [-3, None, 2])
def test_channel_index_offset(offset):
    if offset is not None and offset < 0:
        with pytest.raises(TypeError):
            rd.WorkTable([], 2, 2, offset)
    else:
        t = rd.WorkTable([], 2, 2) if offset is None else rd.WorkTable([], 2, 2, offset)
        assert t.channel_index_offset == (0 if offset is None else offset)


@pytest.mark.parametrize("offsets", [[1], [1, 1], [[1, 1], []], [[1, 1], [1]],
                                     [[1, 1], [1, 1, 1]]])
def test_psfs_wrong_shape(offsets):
    with pytest.raises(TypeError):
        rd.WorkTable(offsets, 1, 1)


def test_add_entries_wrong_type():
    entries = [rd.WorkTableEntry() for _ in range(3)]
    with pytest.raises(TypeError):
        entries[0].psfs.append(np.ones((4, 4), np.float64))
    with pytest.raises(TypeError):
        entries[1].residual = np.ones((4, 4), int)
    with pytest.raises(TypeError):
        entries[2].model = np.ones((4, 4), complex)


def test_add_entries():
    t = rd.WorkTable([], 3, 1)
    entries = [rd.WorkTableEntry() for _ in range(3)]
    img = np.ones((4, 4), np.float32)
    entries[0].psfs.append(img)
    entries[1].residual = img
    entries[2].model = img
    with pytest.raises(AttributeError):
        _ = entries[1].residual
    with pytest.raises(AttributeError):
        _ = entries[1].model
    assert len(t) == 0
    for i, e in enumerate(entries):
        e.image_weight = i
        e.original_channel_index = i % 2
        e.band_end_frequency = float(i + 1) * 1e6
        t.add_entry(e)
    assert len(t) == 3
    assert [len(g) for g in t.original_groups] == [2, 1, 0]
    for i, e in enumerate(t):
        assert e.image_weight == i
        assert e.central_frequency == 0.5 * float(i + 1) * 1e6


def test_str(capsys):
    t = rd.WorkTable([[1, 2], [3, 4], [5, 6]], 0, 0)
    expect = ("=== IMAGING TABLE ===\nOriginal groups       1\nDeconvolution groups  1\n"
              "Channel index         0\n=== PSFs ===\n[x: 1, y: 2]\n[x: 3, y: 4]\n"
              "[x: 5, y: 6]\n")
    assert str(t) == expect
    print(t)
    assert capsys.readouterr().out == expect + "\n"
