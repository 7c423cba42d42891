"""The C-ABI boundary without a GPU: the library loads, exports every symbol include/*.h declares,
its struct layouts match the ctypes mirror, and compute entry points fail loudly (no fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from ripplemq_amd import _abi as A
from ripplemq_amd.engine import Engine, EngineConfig, EngineError

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(A.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    return A.load()


def test_exports_every_header_symbol(lib):
    syms = A.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(A._SIGS), "ctypes signatures must cover exactly the header"


def test_no_torch_or_oracle_in_library(lib):
    out = subprocess.run(["ldd", A.LIB_PATH], capture_output=True, text=True).stdout
    assert "torch" not in out and "ripple_oracle" not in out and "python" not in out
    nm = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True, text=True).stdout
    assert "ro_append" not in nm and "ro_crc32c" not in nm


def test_struct_layouts_match_ctypes(tmp_path):
    exe = tmp_path / "abi_layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), os.path.join(HERE, "abi_layout.c")], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    structs = {"rmq_config": A.RmqConfig, "rmq_batch": A.RmqBatch, "rmq_fetch_req": A.RmqFetchReq,
               "rmq_fetch_res": A.RmqFetchRes, "rmq_partition_state": A.RmqPartitionState,
               "rmq_append_stats": A.RmqAppendStats}
    for k, v in got.items():
        if "." in k:
            s, f = k.split(".")
            assert getattr(structs[s], f).offset == int(v), k
        else:
            assert C.sizeof(structs[k]) == int(v), k


def test_strerror_and_defaults(lib):
    assert lib.rmq_strerror(A.RMQ_ENOTLEADER) == b"Not leader"
    # every status the header declares has its own message
    hdr = open(os.path.join(REPO, "include", "ripplemq_engine.h")).read()
    codes = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"\b(RMQ_(?:OK|PENDING|E[A-Z]+))\s*=\s*(-?\d+)", hdr))
    assert "RMQ_ETERM" in codes and "RMQ_ESTALE" in codes, codes
    msgs = {name: lib.rmq_strerror(v) for name, v in codes.items()}
    assert all(m and m != b"unknown status" for m in msgs.values()), msgs
    assert len(set(msgs.values())) == len(msgs), msgs
    assert lib.rmq_abi_version() == A.RMQ_ABI_VERSION
    c = A.RmqConfig()
    lib.rmq_config_default(C.byref(c), 4096, 3)
    assert c.num_partitions == 4096 and c.replication_factor == 3 and c.index_interval == 1024


def test_invalid_configs_rejected_before_device(lib):
    for kw in [dict(num_partitions=0), dict(num_partitions=4, replication_factor=9),
               dict(num_partitions=4, segment_bytes=3 << 20), dict(num_partitions=4, index_interval=100),
               dict(num_partitions=4, max_batch_records=1 << 30)]:
        with pytest.raises(EngineError) as ei:
            Engine(EngineConfig(**kw))
        assert ei.value.status == A.RMQ_EINVAL


def test_create_without_gpu_fails_loudly(lib):
    try:
        import torch  # noqa: F401 — only to ask whether a GPU exists
        has_gpu = torch.cuda.device_count() > 0
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("a GPU is present")
    with pytest.raises(EngineError) as ei:
        Engine(EngineConfig(num_partitions=4))
    assert ei.value.status == A.RMQ_EDEVICE
    h = C.c_void_p()
    assert lib.rmq_append(None, None, None, None) == A.RMQ_EINVAL
    assert lib.rmq_fetch(None, None, 0, 0, None, 0, None, None) == A.RMQ_EINVAL
    assert not h.value
