"""Transcribes the reference's known-answer vectors into data fixtures under tests/golden/.

Run once in the build container (the only place /root/reference exists):
    python tools/extract_reference_fixtures.py
It reads the reference's JUnit sources as text and writes the (input, expected)
pairs they hold as JSON -- data only, no reference code is copied:
  * MurmurHash3Test.java:27-176  -> 150 x86_32 vectors (string key, seed, expected)
  * MurmurHash3Test.java:181-480 -> 300 x64_64 vectors (string key, seed, expected)
  * MurmurHash3Test.java:485-486 -> 1 binary x64_64 vector (hex key)
  * UtilTest.java:43-87          -> VLQ size table and decode vectors
  * AddressSizeTest.java:16-48   -> LE address byte vectors
  * BytesWrittenTest.java:43-57  -> putSize / deleteSize scenario
"""
import json
import os
import re

REF = "/root/reference/src/test/java/com/spotify/sparkey"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def s32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(os.path.join(REF, "MurmurHash3Test.java")).read()
    x86 = []
    for line_no, line in enumerate(src.splitlines(), 1):
        m = re.search(r'assert_murmurhash3_x86_32\((0x[0-9a-fA-F]+), "([^"]*)", (0x[0-9a-fA-F]+)\);', line)
        if m:
            x86.append({"key": m.group(2), "seed": s32(int(m.group(3), 16)),
                        "expected": int(m.group(1), 16) & 0xFFFFFFFF, "line": line_no})
    x64 = []
    for line_no, line in enumerate(src.splitlines(), 1):
        m = re.search(r'assert_murmurhash3_x64_64\((0x[0-9a-fA-F]+)L, "([^"]*)", (0x[0-9a-fA-F]+)\);', line)
        if m:
            x64.append({"key": m.group(2), "seed": s32(int(m.group(3), 16)),
                        "expected": int(m.group(1), 16) & 0xFFFFFFFFFFFFFFFF, "line": line_no})
    binary = []
    mb = re.search(r'decode\("([0-9a-f]+)"\);\s*assert_murmurhash3_x64_64\((-?\d+)L, decoded, (-?\d+)\);', src)
    if mb:
        line_no = src[:mb.start()].count("\n") + 1
        binary.append({"key_hex": mb.group(1), "seed": s32(int(mb.group(3))),
                       "expected": int(mb.group(2)) & 0xFFFFFFFFFFFFFFFF, "line": line_no})
    json.dump({"source": "src/test/java/com/spotify/sparkey/MurmurHash3Test.java",
               "x86_32": x86, "x64_64": x64, "x64_64_binary": binary},
              open(os.path.join(OUT, "murmur3_kat.json"), "w"), indent=1)

    util = open(os.path.join(REF, "UtilTest.java")).read()
    sizes = []
    for m in re.finditer(r'assertEquals\((\d), Util\.unsignedVLQSize\(([^)]*)\)\);', util):
        expr = m.group(2).strip()
        if expr == "Long.MAX_VALUE":
            val = (1 << 63) - 1
        else:
            mm = re.match(r'1L? << (\d+)', expr)
            val = 1 << int(mm.group(1))
        sizes.append({"value": val, "expected": int(m.group(1))})
    decodes = []
    for m in re.finditer(r'checkVLQ\(\s*(\d+), new byte\[\] \{([^}]*)\}\);', util):
        bs = [int(x, 16) for x in re.findall(r'0x([0-9a-f]{2})', m.group(2))]
        decodes.append({"bytes": bs, "expected": int(m.group(1))})
    too_long = [0xcb, 0xcb, 0xf6, 0xae, 0x89, 0x07]  # UtilTest.java:70-76 (must throw)
    json.dump({"source": "src/test/java/com/spotify/sparkey/UtilTest.java",
               "size": sizes, "decode": decodes, "too_long": [too_long]},
              open(os.path.join(OUT, "vlq_kat.json"), "w"), indent=1)

    addr = {"source": "src/test/java/com/spotify/sparkey/AddressSizeTest.java",
            "long": {"bytes": [1, 2, 3, 4, 5, 6, 7, 8], "value": 0x0807060504030201},
            "int": {"bytes": [1, 2, 3, 4], "value": 0x04030201}}
    bw = open(os.path.join(REF, "BytesWrittenTest.java")).read()
    assert "13 * (17 + 47 + 1 + 1) + 19 * (130 + 32000 + 2 + 3)" in bw
    assert "3 * (130 + 2 + 1)" in bw
    bytes_written = {"source": "src/test/java/com/spotify/sparkey/BytesWrittenTest.java",
                     "puts": [[17, 47, 13], [130, 32000, 19]], "deletes": [[130, 3]],
                     "put_size": 13 * (17 + 47 + 1 + 1) + 19 * (130 + 32000 + 2 + 3),
                     "delete_size": 3 * (130 + 2 + 1)}
    json.dump({"address_size": addr, "bytes_written": bytes_written},
              open(os.path.join(OUT, "format_kat.json"), "w"), indent=1)
    print(f"x86_32={len(x86)} x64_64={len(x64)} binary={len(binary)} vlq_size={len(sizes)} "
          f"vlq_decode={len(decodes)}")


if __name__ == "__main__":
    main()
