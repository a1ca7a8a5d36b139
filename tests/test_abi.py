"""The C-ABI library loads and exports every entry point include/*.h declares
(ksched.h: device evaluator and annotator; ksched_snapshot.h: the native
snapshot encoder), and the ctypes mirrors have the C compiler's layouts."""
import ctypes
import os
import re

from conftest import ROOT, pkg


def declared_symbols():
    out = set()
    inc = os.path.join(ROOT, "include")
    for h in sorted(os.listdir(inc)):
        if h.endswith(".h"):
            src = open(os.path.join(inc, h)).read()
            out |= set(re.findall(r"^\s*(?:int|const char\*)\s+(ksg_\w+)\s*\(", src, re.M))
    return sorted(out)


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("ksg_open", "ksg_eval", "ksg_commit", "ksg_run_queue", "ksg_run_replicas", "ksg_last_error",
              "ksg_append_pods", "ksg_eval_pod", "ksg_snapshot_new", "ksg_snapshot_add_pod", "ksg_snapshot_sync",
              "ksg_snapshot_status", "ksg_snapshot_prefilter"):
        assert s in syms


def test_library_exports_every_symbol(built):
    native = pkg("native")
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    lib.ksg_abi_version.restype = ctypes.c_int
    assert lib.ksg_abi_version() == 4


def test_struct_layouts_match(tmp_path):
    """ctypes / numpy mirrors of the ABI structs have the C compiler's layout."""
    import subprocess
    native = pkg("native")
    E = pkg("encoder")
    src = tmp_path / "sz.c"
    names = ["ksg_nodes", "ksg_topology", "ksg_pod", "ksg_workload", "ksg_profile", "ksg_result",
             "ksg_capture", "ksg_node_state", "ksg_replica_summary", "ksg_kernel_stat", "ksg_names",
             "ksg_annotate_in", "ksg_eval_rows"]
    src.write_text('#include <stdio.h>\n#include "ksched.h"\nint main(void){' +
                   "".join(f'printf("%zu\\n", sizeof({n}));' for n in names) + "return 0;}")
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    sizes = dict(zip(names, map(int, subprocess.check_output([str(exe)]).split())))
    assert sizes["ksg_pod"] == E.POD_DTYPE.itemsize
    assert sizes["ksg_nodes"] == ctypes.sizeof(native.KsgNodes)
    assert sizes["ksg_topology"] == ctypes.sizeof(native.KsgTopology)
    assert sizes["ksg_workload"] == ctypes.sizeof(native.KsgWorkload)
    assert sizes["ksg_profile"] == ctypes.sizeof(native.KsgProfile)
    assert sizes["ksg_result"] == ctypes.sizeof(native.KsgResult) == native.RESULT_DTYPE.itemsize
    assert sizes["ksg_capture"] == ctypes.sizeof(native.KsgCapture)
    assert sizes["ksg_node_state"] == ctypes.sizeof(native.KsgNodeState)
    assert sizes["ksg_replica_summary"] == ctypes.sizeof(native.KsgReplicaSummary)
    assert sizes["ksg_kernel_stat"] == ctypes.sizeof(native.KsgKernelStat)
    assert sizes["ksg_names"] == ctypes.sizeof(native.KsgNames)
    assert sizes["ksg_annotate_in"] == ctypes.sizeof(native.KsgAnnotateIn)
    assert sizes["ksg_eval_rows"] == ctypes.sizeof(native.KsgEvalRows)


def test_snapshot_view_layouts(tmp_path):
    """ctypes mirrors of the ksched_snapshot.h views (snapshot.py)."""
    import subprocess
    S = pkg("snapshot")
    pairs = {"ksg_str_pair": S.StrPair, "ksg_quantity": S.Quantity, "ksg_taint_view": S.TaintView,
             "ksg_toleration_view": S.TolerationView, "ksg_requirement_view": S.RequirementView,
             "ksg_node_selector_term_view": S.NodeSelectorTermView, "ksg_preferred_term_view": S.PreferredTermView,
             "ksg_label_selector_view": S.LabelSelectorView, "ksg_affinity_term_view": S.AffinityTermView,
             "ksg_spread_view": S.SpreadView, "ksg_host_port_view": S.HostPortView, "ksg_container_view": S.ContainerView, "ksg_image_view": S.ImageView,
             "ksg_node_view": S.NodeView, "ksg_volume_view": S.VolumeView, "ksg_pod_view": S.PodView, "ksg_plugin_view": S.PluginView,
             "ksg_plugin_set_view": S.PluginSetView, "ksg_profile_view": S.ProfileView,
             "ksg_profile_info": S.ProfileInfo}
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "ksched_snapshot.h"\nint main(void){' +
                   "".join(f'printf("%zu\\n", sizeof({n}));' for n in pairs) + "return 0;}")
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    sizes = list(map(int, subprocess.check_output([str(exe)]).split()))
    for (n, t), sz in zip(pairs.items(), sizes):
        assert sz == ctypes.sizeof(t), n


def test_product_path_fails_loudly_without_library(tmp_path):
    native = pkg("native")
    import pytest
    with pytest.raises(native.KschedError):
        native.Engine(lib_path=str(tmp_path / "missing.so"))


def test_library_embeds_the_tree_source_hash(built):
    """bench.py measures the committed source: the built library carries the
    sha256 of csrc/ + include/ (ksg_source_hash), equal to the tree's."""
    import importlib
    ge = importlib.import_module("__graft_entry__")
    native = pkg("native")
    lib = ctypes.CDLL(native.LIB_PATH)
    lib.ksg_source_hash.restype = ctypes.c_char_p
    want = ge.source_hash()
    assert lib.ksg_source_hash().decode() == want
    assert ge.library_hash(native.LIB_PATH) == want
