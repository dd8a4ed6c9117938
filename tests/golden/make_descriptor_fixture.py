"""Generates tests/golden/test_message_descriptor.json from data the reference holds.

Source: the serialized FileDescriptorProto that protoc embedded in the reference's generated
test message class, `descriptorData` at
  /root/reference/src/test/java/ir/sahab/kafka/test/proto/TestMessage.java:750-755
(the compiled form of src/test/resources/test-message.proto:1-10).  That Java string literal
is un-escaped to its bytes (protoc writes each byte as a Latin-1 char: octal escapes for the
non-printables), parsed with google.protobuf's own descriptor_pb2, and stored as data:

  file_descriptor_hex   the FileDescriptorProto bytes, verbatim
  message_full_name     Descriptor.getFullName()            -> Parquet schema name
  proto_class           Java class of the message            -> "parquet.proto.class"
  columns               (name, number, type, label) per field in declaration order
                        (what ProtoSchemaConverter turns into the Parquet schema)
  descriptor_text       TextFormat.printToString(descriptor.toProto()), the value
                        parquet-protobuf 1.10.1 ProtoWriteSupport.serializeDescriptor puts
                        under "parquet.proto.descriptor" (google.protobuf's text_format
                        prints the same field order, indentation and enum names)

Only the bytes are read from the reference (study-only text); no reference source is copied.
Run in the build container (the reference is not on the GPU box):
  python tests/golden/make_descriptor_fixture.py
"""
import json
import os
import re

from google.protobuf import descriptor_pb2, text_format

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/test/java/ir/sahab/kafka/test/proto/TestMessage.java"
OUT = os.path.join(HERE, "test_message_descriptor.json")


def java_string_bytes(lit):
    """Bytes of a protoc-emitted Java string literal body (chars are Latin-1 bytes)."""
    out = bytearray()
    i = 0
    simple = {"n": 10, "t": 9, "r": 13, "b": 8, "f": 12, '"': 34, "'": 39, "\\": 92}
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out.append(ord(c))
            i += 1
            continue
        d = lit[i + 1]
        if d in simple:
            out.append(simple[d])
            i += 2
        elif d in "01234567":
            m = re.match(r"[0-7]{1,3}", lit[i + 1:])
            out.append(int(m.group(0), 8))
            i += 1 + len(m.group(0))
        elif d == "u":
            out.append(int(lit[i + 2:i + 6], 16))
            i += 6
        else:
            raise ValueError("escape \\%s" % d)
    return bytes(out)


def main():
    src = open(REF, encoding="utf-8").read()
    block = src[src.index("descriptorData = {"):]
    block = block[:block.index("};")]
    parts = re.findall(r'"((?:[^"\\]|\\.)*)"', block)
    fdp_bytes = b"".join(java_string_bytes(p) for p in parts)
    fdp = descriptor_pb2.FileDescriptorProto.FromString(fdp_bytes)
    assert len(fdp.message_type) == 1
    msg = fdp.message_type[0]
    full_name = (fdp.package + "." if fdp.package else "") + msg.name
    outer = fdp.options.java_package + "." + fdp.options.java_outer_classname
    fixture = {
        "source": "TestMessage.java:750-755 descriptorData (protoc-generated from test-message.proto:1-10)",
        "file_descriptor_hex": fdp_bytes.hex(),
        "file_name": fdp.name,
        "message_full_name": full_name,
        "proto_class": outer + "$" + msg.name,
        "columns": [[f.name, f.number, f.type, f.label] for f in msg.field],
        "descriptor_text": text_format.MessageToString(msg),
    }
    json.dump(fixture, open(OUT, "w"), indent=1)
    print("wrote", OUT)
    print(fixture["descriptor_text"])


if __name__ == "__main__":
    main()
