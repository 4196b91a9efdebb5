"""The INTEGRATION.md ctypes stub against the built library (CPU: no kernel
launch).  Loading the stub runs its own struct-size assertion against
cmt_attn_args_size(); this test also pins it to native.AttnArgs."""
import ctypes

from _stub import load_stub


def test_stub_struct_matches_library():
    from projects.mmdet3d_plugin import native
    ns = load_stub()
    L = native.lib()
    assert ctypes.sizeof(ns["_AttnArgs"]) == L.cmt_attn_args_size() == ctypes.sizeof(native.AttnArgs)
    assert [f[0] for f in ns["_AttnArgs"]._fields_] == [f[0] for f in native.AttnArgs._fields_]


def test_every_struct_mirror_matches_library():
    from projects.mmdet3d_plugin import native
    L = native.lib()
    for name, st in native.STRUCTS.items():
        assert getattr(L, f"cmt_{name}_args_size")() == ctypes.sizeof(st), name


def test_chain_workspace_size_export():
    from projects.mmdet3d_plugin import native
    L = native.lib()
    for rows in (1, 31, 32, 33, 900, 1800, 3000):
        assert L.cmt_chain_ws_bytes(rows) == 4 * native.chain_ws_numel(rows)
    assert L.cmt_chain_ws_bytes(900) == 4 * 4 * 29 * 32 * 256   # whole 32-row tiles, not 4 * rows * 256
