"""The substep-queue kernel, the list tiers and the per-env-step kernels read their own arguments through __builtin_amdgcn_kernarg_segment_ptr() as a
WQArgs struct (ur3e_batch.hip, W_KARG_PTR: fields loaded where used instead of all at entry, which had kept
560 bytes of KConfig / KState in SGPRs and spilled 256 of them).  That is only right while the compiler lays
the explicit kernel arguments out as C lays out a struct of the same members: each at the next offset
aligned to its size's natural alignment, from 0.  The host compile checks WQArgs against that rule
(static_assert); this test checks the rule against the code object's kernarg metadata of every queue kernel
of the built library (CPU only, no GPU)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "ur3e_amd", "_lib", "libur3e_amd.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
@pytest.mark.parametrize("prefix,nargs", [("_Z12w_env_step_q", 18), ("_Z15w_env_step_list", 21),
                                          ("_Z10w_env_stepI", 13)])
def test_kernel_kernarg_layout_is_the_struct_layout(prefix, nargs):
    """the queue kernel (WQArgs), the list tiers (WLArgs) and the per-env-step kernels (WEArgs)"""
    from ur3e_amd.codeobj import kernels
    qs = [k for k in kernels(LIB) if k.get("name", "").startswith(prefix)]
    assert qs, f"no {prefix} kernel in the library"
    for k in qs:
        args = [a for a in k["args"] if not str(a.get("value_kind", "")).startswith("hidden")]
        assert len(args) == nargs, (k["name"], len(args))
        off = 0
        for a in args:
            size = a["size"]
            align = 8 if size >= 8 else size  # by-value structs of this ABI carry 8-byte members
            off = (off + align - 1) // align * align
            assert a["offset"] == off, (k["name"], args)
            off += size
        # KConfig and KState by value at 16 and 16 + sizeof(KConfig), as WQArgs places them
        assert args[2]["value_kind"] == "by_value" and args[2]["offset"] == 16
        assert args[3]["value_kind"] == "by_value" and args[3]["offset"] == 16 + args[2]["size"]
