"""Writes tests/golden/spec_vectors.json: hand-derived known-answer vectors.

RLE/bit-packing hybrid (parquet-format Encodings.md "RLE"): values are packed LSB-first
(the spec's own example: 0..7 at bit width 3 -> 0x88 0xC6 0xFA); bit-packed runs carry a
(groups << 1 | 1) header and hold at most 63 groups in parquet-mr's encoder; an RLE run
needs >= 8 repeats starting on a group boundary; the last partial group is zero padded.
Each expected byte string below was derived by hand (bit tables in the comments), NOT by
running any encoder in this repository.
"""
import json
import os

V = []


def add(name, values, width, hexbytes, note):
    V.append({"name": name, "values": values, "bit_width": width, "expected_hex": hexbytes.replace(" ", ""),
              "note": note})


add("spec_0_to_7_w3", list(range(8)), 3, "03 88 C6 FA", "Encodings.md example; one bit-packed group")
add("rle_10x4_w3", [4] * 10, 3, "14 04", "varint(10<<1)=0x14, value in 1 byte")
add("w0_5_zeros", [0] * 5, 0, "03", "width 0: partial group -> bit-packed header only")
add("w0_20_zeros", [0] * 20, 0, "28", "width 0: RLE run of 20, no value bytes")
add("bp_then_rle_w3", [1, 2, 3, 4, 5, 6, 7, 7] + [7] * 8, 3, "03 D1 58 FF 10 07",
    "group [1..7,7] packed D1 58 FF; repeats inside a packed group do not count; then RLE(8,7)")
add("rle_then_realign_w3", [5] * 10 + [1, 2, 3, 4, 5, 6, 7, 0], 3, "14 05 03 D1 58 1F",
    "RLE(10,5) then a group realigned at index 10: [1..7,0] -> D1 58 1F")
add("swallowed_repeats_w3", [1, 2, 3, 4, 5] + [6] * 9, 3, "05 D1 58 DB B6 6D 03",
    "[1,2,3,4,5,6,6,6] -> D1 58 DB; six trailing 6s < 8 -> padded group [6x6,0,0] -> B6 6D 03; 2 groups")
add("split_63_groups_w1", [i % 2 for i in range(512)], 1, "7F" + "AA" * 63 + "03AA",
    "64 bit-packed groups: a run of 63 (header 0x7F) then a run of 1")
add("rle_300_w1", [1] * 300, 1, "D8 04 01", "varint(600) = D8 04")
add("rle_w8", [255] * 8, 8, "10 FF", "exactly 8 repeats -> RLE")
add("rle_w9", [300] * 8, 9, "10 2C 01", "value padded to ceil(9/8)=2 bytes LE")
add("rle_w32", [0xDEADBEEF] * 9, 32, "12 EF BE AD DE", "width 32")
add("empty", [], 3, "", "no values -> no bytes")
add("seven_equal_w2", [3] * 7, 2, "03 FF 3F", "7 repeats < 8 -> padded bit-packed group")

SNAPPY = [
    {"name": "one_byte", "input_hex": "61", "expected_hex": "010061", "note": "varint(1), literal tag 0"},
    {"name": "aaaa24", "input_hex": "61" * 24, "expected_hex": "180061" + "5A0100",
     "note": "literal 'a' then COPY_2_BYTE_OFFSET len 23 off 1 (tag 2+(22<<2)=0x5A)"},
    {"name": "short14", "input_hex": "6162636465666768696a6b6c6d6e", "expected_hex": "0e34" + "6162636465666768696a6b6c6d6e",
     "note": "< kInputMarginBytes: single literal, tag (13<<2)=0x34"},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spec_vectors.json")
    with open(out, "w") as f:
        json.dump({"rle_hybrid": V, "snappy": SNAPPY}, f, indent=1)
    print("wrote", out, len(V), "rle vectors", len(SNAPPY), "snappy vectors")
