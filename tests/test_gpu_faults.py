"""The writer's sticky failure path under real I/O failures (file mode, fwrite on the assembly
thread).  The reference retries close() forever on IOException (tryUntilSucceeds,
KafkaProtoParquetWriter.java:327-336,410-428) and parquet-mr's close() re-runs the flush while
`closed` is false, so after a failed flush:
  - close() returns non-zero, and a retried close() again returns non-zero (never a silent
    success over a short file);
  - every later write / getDataSize reports the failure;
  - getNumWrittenRecords() never counts a record whose write() did not return success.
Failures are real: RLIMIT_FSIZE makes the kernel refuse writes past a byte position
(SIGXFSZ ignored, so write(2) returns EFBIG) mid-file, and /dev/full fails the first flush
(ENOSPC).  No test hook in the library."""
import contextlib
import os
import resource
import signal

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
MiB = 1024 * 1024


@contextlib.contextmanager
def file_size_limit(nbytes):
    """RLIMIT_FSIZE soft limit for this process (restored after); SIGXFSZ ignored."""
    soft, hard = resource.getrlimit(resource.RLIMIT_FSIZE)
    old = signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
    resource.setrlimit(resource.RLIMIT_FSIZE, (nbytes, hard))
    try:
        yield
    finally:
        resource.setrlimit(resource.RLIMIT_FSIZE, (soft, hard))
        signal.signal(signal.SIGXFSZ, old)


def _writer(path, block_size):
    import kpw
    props = kpw.ParquetProperties(block_size=block_size, compression_codec_name=kpw.SNAPPY)
    return kpw.ParquetFile(path, kpw.Schema(synth.REC8.message_name, synth.REC8.columns, synth.REC8.proto_class),
                           props)


def _after_failure(pf, accepted):
    """close() fails and keeps failing; counts never exceed what write() accepted."""
    import kpw
    L = pf._L
    st1 = L.kpw_writer_close(pf._h)
    st2 = L.kpw_writer_close(pf._h)
    assert st1 != 0 and st2 != 0, (st1, st2)
    assert L.kpw_writer_data_size(pf._h) == -1
    assert 0 <= pf.get_num_written_records() <= accepted
    with pytest.raises(kpw.KpwError):
        pf.write_batch([b"\x08\x01"])
    assert pf.get_num_written_records() <= accepted


@pytest.mark.parametrize("mode", ["bulk", "per_record"])
def test_write_failure_mid_file(tmp_path, mode):
    """The file system refuses bytes past 3 MiB: the row groups before it reach the file, the
    one that crosses it fails on the assembly thread; the failure is sticky."""
    data, offs = synth.generate(synth.KIND_REC8, 0xFA17, 400_000 if mode == "bulk" else 150_000)
    path = str(tmp_path / "f.parquet")
    pf = _writer(path, 1 * MiB)
    accepted = 0
    failed_at = None
    n = len(offs) - 1
    with file_size_limit(3 * MiB):
        if mode == "bulk":
            step = 70_000   # > 65536: GPU-planned jobs
            for a in range(0, n, step):
                b = min(n, a + step)
                try:
                    pf.write_batch((data[int(offs[a]):int(offs[b])], (offs[a:b + 1] - offs[a]).astype(np.uint64)))
                    accepted += b - a
                except Exception:  # noqa: BLE001
                    failed_at = a
                    break
                if pf._L.kpw_writer_data_size(pf._h) < 0:   # the failure surfaced at getDataSize
                    failed_at = b
                    break
        else:
            L = pf._L
            one = np.zeros(2, dtype=np.uint64)
            for i in range(n):
                a, b = int(offs[i]), int(offs[i + 1])
                one[1] = b - a
                if L.kpw_writer_write(pf._h, data.ctypes.data + a, one.ctypes.data, 1) != 0:
                    failed_at = i
                    break
                accepted += 1
                if L.kpw_writer_data_size(pf._h) < 0:   # the failure surfaced at getDataSize
                    failed_at = i
                    break
        _after_failure(pf, accepted)
    assert os.path.getsize(path) <= 3 * MiB
    assert failed_at is not None or accepted == n
    pf.__del__()


def test_write_failure_dev_full():
    """/dev/full: the first flush of buffered bytes fails (ENOSPC); close() reports it."""
    if not os.path.exists("/dev/full"):
        pytest.skip("no /dev/full")
    data, offs = synth.generate(synth.KIND_REC8, 0xFA18, 120_000)
    pf = _writer("/dev/full", 1 * MiB)
    try:
        pf.write_batch((data, offs))
        accepted = len(offs) - 1
    except Exception:  # noqa: BLE001
        accepted = 0
    _after_failure(pf, accepted)
    pf.__del__()


def test_close_retry_after_success_is_idempotent(tmp_path):
    """The other half of the contract: a successful close() stays successful on retry and
    does not append a second footer."""
    data, offs = synth.generate(synth.KIND_REC8, 0xFA19, 50_000)
    path = str(tmp_path / "ok.parquet")
    pf = _writer(path, 1 * MiB)
    pf.write_batch((data, offs))
    assert pf._L.kpw_writer_close(pf._h) == 0
    size = os.path.getsize(path)
    assert pf._L.kpw_writer_close(pf._h) == 0
    assert os.path.getsize(path) == size
    assert pf.get_num_written_records() == len(offs) - 1
    pf.__del__()
