"""Proto2 wire edge cases of the reference's parse step, shared by the oracle tests
(test_oracle.py) and the HIP decode tests (test_gpu_wire.py).

The semantics are protobuf-java's generated parse loop for the reference's test message
(src/test/java/ir/sahab/kafka/test/proto/TestMessage.java:85-139: switch on the full tag,
default -> parseUnknownField; last occurrence of a field wins) plus isInitialized
(:263-278, a missing required field makes parseFrom throw), reached from
KafkaProtoParquetWriter.java:268-276.
"""
import protoutil
import synth


def varint(v):
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def tag(f, wt):
    return varint((f << 3) | wt)


def sample_msg(**kw):
    cls = protoutil.message_class(synth.SAMPLE)
    m = cls()
    for k, v in kw.items():
        setattr(m, k, v)
    return m


def accepted():
    """Records parseFrom accepts: (label, bytes)."""
    base = sample_msg(query="q", timestamp=7).SerializeToString()
    return [
        ("canonical", base),
        ("negative_int32_10_byte_varint", sample_msg(query="a", timestamp=1, page_number=-5).SerializeToString()),
        ("unknown_varint_and_len", base + tag(99, 0) + varint(12345) + tag(98, 2) + varint(3) + b"xyz"),
        ("last_occurrence_wins", base + tag(2, 0) + varint(42)),
        ("reordered_fields", tag(4, 0) + varint(9) + tag(2, 0) + varint(3) + tag(1, 2) + b"\x02hi"),
        ("nested_unknown_groups", base + tag(50, 3) + tag(51, 0) + varint(1) + tag(52, 3) + tag(53, 5) + b"wxyz" +
         tag(52, 4) + tag(50, 4)),
        ("known_number_foreign_wire_type", base + tag(3, 2) + b"\x01z"),
        ("unknown_fixed32_fixed64", base + tag(60, 5) + b"abcd" + tag(61, 1) + b"12345678"),
        ("zero_and_empty_values", sample_msg(query="", timestamp=0, page_number=0, result_per_page=-1).SerializeToString()),
        ("string_repeated_last_wins", tag(1, 2) + b"\x03abc" + tag(2, 0) + varint(5) + tag(1, 2) + b"\x02de"),
        ("optional_repeated_last_wins", base + tag(3, 0) + varint(11) + tag(4, 0) + varint(2) + tag(3, 0) + varint(12)),
        ("max_varints", tag(1, 2) + b"\x01m" + tag(2, 0) + varint((1 << 64) - 1) + tag(3, 0) + varint((1 << 64) - 1)),
        ("int32_from_wide_varint", tag(1, 2) + b"\x01w" + tag(2, 0) + varint(1 << 62) + tag(4, 0) + varint((1 << 40) + 7)),
        ("unknown_field_number_above_1023", base + tag(5000, 0) + varint(1) + tag((1 << 29) - 1, 2) + b"\x00"),
        ("long_unknown_len", base + tag(70, 2) + varint(300) + bytes(range(256)) + bytes(44)),
        ("deep_unknown_groups", base + b"".join(tag(80 + i, 3) for i in range(40)) +
         b"".join(tag(80 + i, 4) for i in reversed(range(40)))),
    ]


def invalid():
    """Records parseFrom rejects (InvalidProtocolBufferException / missing required):
    (label, bytes)."""
    q = tag(1, 2) + b"\x01a"
    return [
        ("missing_required_query", tag(2, 0) + varint(1)),
        ("truncated_length_delimited", tag(1, 2) + b"\x05ab"),
        ("truncated_varint", q + tag(2, 0) + b"\x80"),
        ("varint_over_10_bytes", q + tag(2, 0) + b"\x80" * 10 + b"\x01"),
        ("wire_type_6", q + tag(2, 0) + varint(1) + tag(7, 6)),
        ("field_number_0", q + tag(2, 0) + varint(1) + b"\x00"),
        ("stray_end_group", q + tag(2, 0) + varint(1) + tag(9, 4)),
        ("mismatched_end_group", q + tag(2, 0) + varint(1) + tag(9, 3) + tag(8, 4)),
        ("required_as_fixed64_is_unknown", q + tag(2, 1) + b"\x01\x02"),
    ]
