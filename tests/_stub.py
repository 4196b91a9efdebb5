"""Loads the reference-side ctypes stub of INTEGRATION.md section 3 verbatim
(the python block between the stub markers) so the tests execute exactly the
text a maintainer would paste into the reference's attention.py."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cmt-cooperative-perception_amd", "lib", "libcmt_hip.so")


def stub_source():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        text = f.read()
    block = re.search(r"<!-- stub:begin -->\s*```python\n(.*?)```\s*<!-- stub:end -->", text, re.S)
    assert block, "INTEGRATION.md lost its stub markers"
    return block.group(1)


def load_stub():
    os.environ.setdefault("CMT_HIP_LIB", LIB)
    ns = {"__name__": "reference_attention_stub"}
    exec(compile(stub_source(), "INTEGRATION.md:stub", "exec"), ns)
    return ns
