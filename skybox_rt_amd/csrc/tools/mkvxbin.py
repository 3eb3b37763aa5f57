#!/usr/bin/env python3
"""Wrap a gfx950 code object into a Vortex kernel image (.vxbin).

Layout follows the reference's kernel/scripts/vxbin.py:54-78: a 16-byte
little-endian header {min_vma, max_vma} followed by the image.  Here the image
is the HIP code object, `min_vma` is where vx_upload_kernel_bytes() reserves
it in the device address space, and max_vma - min_vma is its reserved size.
"""
import struct
import sys


def main(argv):
    if len(argv) != 4:
        print("usage: mkvxbin.py <code_object> <min_vma> <out.vxbin>", file=sys.stderr)
        return 2
    src, vma, dst = argv[1], int(argv[2], 0), argv[3]
    img = open(src, "rb").read()
    size = (len(img) + 4095) & ~4095
    with open(dst, "wb") as f:
        f.write(struct.pack("<QQ", vma, vma + size))
        f.write(img)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
