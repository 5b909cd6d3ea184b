"""Extract the gfx950 code object(s) embedded in a HIP shared library (clang offload bundle
in the .hip_fatbin section) so llvm-objdump can disassemble them:

    python tools/extract_co.py 3d-pose-baseline_amd/libp3d.so /tmp/p3d_gfx950.co
    /opt/rocm/lib/llvm/bin/llvm-objdump -d /tmp/p3d_gfx950.co > /tmp/p3d.s
"""
import struct
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def bundles(blob):
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            o, size, tl = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            yield triple, blob[pos + o:pos + o + size]
        pos = blob.find(MAGIC, pos + 24)


def main(src, dst):
    blob = open(src, "rb").read()
    k = 0
    for triple, data in bundles(blob):
        if "gfx950" in triple and data[:4] == b"\x7fELF":
            out = dst if k == 0 else "%s.%d" % (dst, k)
            open(out, "wb").write(data)
            print(triple, len(data), "->", out)
            k += 1
    if k == 0:
        raise SystemExit("no gfx950 code object found in %s" % src)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
