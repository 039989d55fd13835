"""CPU-side checks of the C-ABI library: it loads, exports every symbol the
headers in include/ declare, and its host logic (index file I/O, properties,
object access, error convention) behaves like the reference.  No compute
call is made here: without a GPU every search must fail loudly."""
import filecmp
import os
import re

import numpy as np
import pytest

import ngt_amd
import ngt_files as F
from ngt_amd import base

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def header_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src)
    skip = {"if", "defined", "sizeof", "return"}
    return sorted({n for n in names if n.startswith(("ngt_", "ngtqg_")) and n not in skip})


@pytest.mark.parametrize("hdr", ["include/ngt_amd.h", "include/NGT/Capi.h", "include/NGT/NGTQ/Capi.h"])
def test_library_exports_every_declared_symbol(hdr):
    L = ngt_amd.lib()
    names = header_functions(os.path.join(ROOT, hdr))
    assert len(names) >= 7
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_open_reads_reference_index_files():
    ix = base.Index(os.path.join(GOLD, "c1_anng"))
    assert ix.dim == 128 and ix.is_float and ix.distance_type == 1
    rows, valid = F.read_obj(os.path.join(GOLD, "c1_anng", "obj"), 128, np.float32)
    for i in [1, 2, 777, 5000]:
        assert np.array_equal(np.array(ix.get_object(i), np.float32), rows[i, :128])
    offs, ids, dists = F.read_grp(os.path.join(GOLD, "c1_anng", "grp"))
    for i in [1, 100, 4999]:
        e = ix.get_edges(i)
        assert [x.id for x in e] == list(ids[offs[i]:offs[i + 1]])
        assert np.array_equal(np.array([x.distance for x in e], np.float32), dists[offs[i]:offs[i + 1]])
    assert ngt_amd.lib().ngt_get_object_repository_size(ix.index, ix.err) == 5001
    ix.close()


def test_save_round_trips_byte_identical(tmp_path):
    for name in ["c1_anng", "c1_onng"]:
        ix = base.Index(os.path.join(GOLD, name))
        out = str(tmp_path / name)
        ix.save(out)
        for f in ["obj", "grp", "tre"]:
            assert filecmp.cmp(os.path.join(GOLD, name, f), os.path.join(out, f), shallow=False), (name, f)
        assert F.read_prf(os.path.join(out, "prf"))["EdgeSizeForSearch"] == \
            F.read_prf(os.path.join(GOLD, name, "prf"))["EdgeSizeForSearch"]
        ix.close()


def test_error_convention():
    L = ngt_amd.lib()
    err = L.ngt_create_error_object()
    assert not L.ngt_open_index(b"/nonexistent/index", err)
    msg = L.ngt_get_error_string(err).decode()
    assert msg.startswith("Capi : ngt_open_index() : Error:")
    L.ngt_clear_error_string(err)
    assert L.ngt_get_error_string(err).decode() == ""
    # parameter errors (Capi.cpp:347-352)
    assert not L.ngt_search_index(None, None, 0, 10, 0.1, -1.0, None, err)
    assert "parametor error" in L.ngt_get_error_string(err).decode()
    L.ngt_destroy_error_object(err)


def test_property_accessors():
    L = ngt_amd.lib()
    err = L.ngt_create_error_object()
    p = L.ngt_create_property(err)
    assert L.ngt_set_property_dimension(p, 96, err)
    assert L.ngt_get_property_dimension(p, err) == 96
    assert L.ngt_set_property_object_type_integer(p, err)
    assert L.ngt_is_property_object_type_integer(L.ngt_get_property_object_type(p, err))
    assert L.ngt_set_property_distance_type_hamming(p, err)
    assert L.ngt_get_property_distance_type(p, err) == 2
    assert L.ngt_set_property_edge_size_for_search(p, 33, err)
    assert L.ngt_get_property_edge_size_for_search(p, err) == 33
    assert L.ngt_get_property_dimension(None, err) == -1
    L.ngt_destroy_property(p)
    L.ngt_destroy_error_object(err)


def test_no_gpu_means_loud_failure():
    if ngt_amd.device_count() > 0:
        pytest.skip("a GPU is present")
    ix = base.Index(os.path.join(GOLD, "c1_anng"))
    q = np.load(os.path.join(GOLD, "queries.npy"))[0].astype(np.float64)
    with pytest.raises(ngt_amd.NativeError) as e:
        ix.search(q, 10, 0.1)
    assert "no HIP device" in str(e.value)
    ix.close()


def test_edge_size_resolution_matches_getEdgeSize():
    # NeighborhoodGraph::getEdgeSize (Graph.h:675-692); host logic, no device needed
    if ngt_amd.device_count() == 0:
        pytest.skip("ngt_amd_index_create needs a device")


def test_ngtqg_host_conventions():
    """ngtqg_* defaults and error convention (NGTQ/Capi.cpp:40-131) without a device."""
    import ctypes
    from ngt_amd._sigs import NGTQGQuantizationParameters, NGTQGQuery
    L = ngt_amd.lib()
    q = NGTQGQuery()
    L.ngtqg_initialize_query(ctypes.byref(q))
    assert (q.size, round(q.epsilon, 6), q.result_expansion) == (20, 0.03, 3.0)
    assert q.radius == np.float32(3.402823466e38)
    p = NGTQGQuantizationParameters()
    L.ngtqg_initialize_quantization_parameters(ctypes.byref(p))
    assert (p.dimension_of_subvector, p.max_number_of_edges) == (0.0, 128)
    err = L.ngt_create_error_object()
    assert not L.ngtqg_open_index(b"/nonexistent/index", err)
    assert L.ngt_get_error_string(err).decode().startswith("Capi : ngtqg_open_index() : Error:")
    assert not L.ngtqg_search_index(None, q, None, err)
    assert "ngtqg_search_index() : parametor error" in L.ngt_get_error_string(err).decode()
    L.ngtqg_close_index(None)
    L.ngt_destroy_error_object(err)


def test_wrong_query_length_rejected():
    """A query whose length is not the index dimension is an error, as
    allocateObject's check makes it (ObjectRepository.h:228-233), on every
    search entry point -- raised before any device work."""
    from ngt_amd import NativeError
    ix = base.Index(os.path.join(GOLD, "c1_anng"))
    with pytest.raises(NativeError):
        ix.batch_search(np.zeros((2, 127), np.float32), 10, 0.1)
    with pytest.raises(NativeError):
        ix.batch_linear_search(np.zeros((2, 129), np.float32), 10)
    with pytest.raises(NativeError, match="dimension"):
        ix.search(np.zeros(129), 10, 0.1)
    with pytest.raises(NativeError, match="dimension"):
        ix.linear_search(np.zeros(100), 10)
    ix.close()
