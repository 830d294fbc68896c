"""``keytab-fix`` (native/keytab/keytab_fix.cpp), the counterpart of the reference's hdfs keytab-fix
tool (frameworks/hdfs/keytab-fix/.../KeytabFix.java:7, Keytab.java, KeytabEntry.java) that every
Kerberized hdfs task runs (frameworks/hdfs/src/main/dist/svc.yml:75-76, HADOOP-16283).

Synthetic MIT keytabs (``testing.keytab``) go in; the rewritten ``hdfs.keytab`` is compared byte
for byte with the expected layout: records without the trailing 32-bit kvno, grouped by principal
in first-appearance order, version 0x0502. Runs against the release and the ASan/UBSan builds.
"""
import os
import subprocess

import pytest

from dcos_commons_amd.testing import keytab as K

P1 = ("LOCAL", ["hdfs", "name-0-node.hdfs.autoip.dcos.thisdcos.directory"])
P2 = ("LOCAL", ["HTTP", "name-0-node.hdfs.autoip.dcos.thisdcos.directory"])


@pytest.fixture(scope="module", params=["release", "sanitize"])
def tool(request):
    from dcos_commons_amd.ops import build

    try:
        targets = build.build_cpp_tools(sanitize=request.param == "sanitize")
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native toolchain unavailable: {e}")
    return [t for t in targets if t.endswith("keytab-fix")][0]


def _run(tool, cwd, *args):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    return subprocess.run([tool, *args], cwd=cwd, capture_output=True, text=True, timeout=30, env=env)


def _entry(p, key, **kw):
    return K.KeytabEntry(p[0], list(p[1]), key, **kw)


def test_rewrites_mit_keytab_for_hadoop(tool, tmp_path):
    k1, k2, k3, k4 = (bytes([i]) * 32 for i in range(1, 5))
    src = [
        _entry(P1, k1, kvno=1, kvno32=1),                              # MIT trailer, same kvno
        _entry(P2, k2, kvno=1, enctype=K.AES128_CTS_HMAC_SHA1_96, kvno32=1),
        _entry(P1, k3, kvno=44, kvno32=300),                           # 32-bit kvno wins, written as u8
        _entry(P2, k4, kvno=2, kvno32=0, padding=b"\0" * 6),           # zero trailer + padding ignored
    ]
    (tmp_path / "secrets-hdfs.keytab").write_bytes(K.encode(src, holes=((2, 12),)))   # and a deleted hole
    r = _run(tool, tmp_path, "secrets-hdfs.keytab")
    assert r.returncode == 0, r.stderr
    assert "Fixing KeyTab File...secrets-hdfs.keytab" in r.stdout and "hdfs.keytab" in r.stdout
    expected = K.encode([
        _entry(P1, k1, kvno=1), _entry(P1, k3, kvno=300 & 0xFF),
        _entry(P2, k2, kvno=1, enctype=K.AES128_CTS_HMAC_SHA1_96), _entry(P2, k4, kvno=2)])
    out = (tmp_path / "hdfs.keytab").read_bytes()
    assert out == expected
    assert all(e.kvno32 is None for e in K.decode(out).entries)   # nothing Hadoop 3.2.0 trips on


def test_v0501_keytab_is_written_as_v0502(tool, tmp_path):
    (tmp_path / "old.keytab").write_bytes(K.encode([_entry(P1, b"k" * 16)], version=0x0501))
    assert _run(tool, tmp_path, "old.keytab").returncode == 0
    assert (tmp_path / "hdfs.keytab").read_bytes() == K.encode([_entry(P1, b"k" * 16)])


def test_empty_component_and_keyless_records(tool, tmp_path):
    src = [_entry(("LOCAL", ["hdfs", ""]), b"a" * 16), _entry(P1, b"", enctype=0)]
    (tmp_path / "k.keytab").write_bytes(K.encode(src))
    r = _run(tool, tmp_path, "k.keytab")
    assert r.returncode == 0 and "dropped 1 record" in r.stderr
    # the reference reads a zero-length component as null and writes the text "null"
    assert (tmp_path / "hdfs.keytab").read_bytes() == K.encode([_entry(("LOCAL", ["hdfs", "null"]), b"a" * 16)])


def test_errors(tool, tmp_path):
    assert _run(tool, tmp_path).returncode == 1
    r = _run(tool, tmp_path, "missing.keytab")
    assert r.returncode == 1 and "does not exist" in r.stderr
    (tmp_path / "bad.keytab").write_bytes(b"\x04\x01rest")
    assert _run(tool, tmp_path, "bad.keytab").returncode == 1
    good = K.encode([_entry(P1, b"k" * 32)])
    (tmp_path / "trunc.keytab").write_bytes(good[:-5])
    assert _run(tool, tmp_path, "trunc.keytab").returncode == 1
    assert not (tmp_path / "hdfs.keytab").exists()


def test_hdfs_kerberos_tasks_run_keytab_fix():
    """The repo's hdfs package fetches the tool and runs it before every Kerberized node starts,
    as the reference's svc.yml does with its jar (svc.yml:75-76)."""
    from dcos_commons_amd.models import hdfs as H
    from dcos_commons_amd.testing import ServiceTestRunner

    r = ServiceTestRunner.for_framework("hdfs")
    for pod in ("journal", "name", "data"):
        r.set_pod_env(pod, SERVICE_ZK_ROOT="/dcos-service-hdfs", DECODED_AUTH_TO_LOCAL="")
    res = (r.set_custom_validators([H.HDFSZoneValidator()])
           .set_options("service.security.kerberos.enabled", "true",
                        "service.security.kerberos.keytab_secret", "__dcos_base64___keytab")
           .run())
    for pod in res.service_spec.pods:
        assert [s.file_path for s in pod.secrets] == ["secrets-hdfs.keytab"]
        assert any(u.endswith("keytab-fix.tar.gz") for u in pod.uris), pod.uris
        for t in pod.tasks:
            assert "./keytab-fix secrets-hdfs.keytab" in t.command.value, (pod.type, t.name)
