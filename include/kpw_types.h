/*
 * kpw_types.h — plain-data types shared by the C-ABI (kpw_gpu.h) and by the CPU
 * oracle (oracle/kpw_oracle.h).  No functions, no torch/HIP types.
 *
 * These describe exactly what the reference's drop-in seam receives:
 *   - the proto2 message schema handed to ParquetFile(Path, Class<T>, ParquetProperties)
 *     (reference src/main/java/ir/sahab/kafka/reader/ParquetFile.java:36-54, converted
 *     to a Parquet schema by parquet-protobuf ProtoSchemaConverter, pinned at
 *     parquet-mr 1.10.1 by reference pom.xml:44-48);
 *   - ParquetProperties(hadoopConf, blockSize, codec, pageSize, enableDictionary)
 *     (ParquetFile.java:105-122) plus the parquet-mr 1.10.1 builder defaults the
 *     reference never overrides (ParquetFile.java:42-50).
 */
#ifndef KPW_TYPES_H
#define KPW_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* google/protobuf/descriptor.proto FieldDescriptorProto.Type numbering, so a host
 * can fill this straight from Descriptors.FieldDescriptor.toProto(). */
enum kpw_proto_type {
    KPW_PT_DOUBLE = 1,  KPW_PT_FLOAT = 2,   KPW_PT_INT64 = 3,    KPW_PT_UINT64 = 4,
    KPW_PT_INT32 = 5,   KPW_PT_FIXED64 = 6, KPW_PT_FIXED32 = 7,  KPW_PT_BOOL = 8,
    KPW_PT_STRING = 9,  KPW_PT_GROUP = 10,  KPW_PT_MESSAGE = 11, KPW_PT_BYTES = 12,
    KPW_PT_UINT32 = 13, KPW_PT_ENUM = 14,   KPW_PT_SFIXED32 = 15, KPW_PT_SFIXED64 = 16,
    KPW_PT_SINT32 = 17, KPW_PT_SINT64 = 18
};

/* FieldDescriptorProto.Label numbering. */
enum kpw_proto_label { KPW_LABEL_OPTIONAL = 1, KPW_LABEL_REQUIRED = 2, KPW_LABEL_REPEATED = 3 };

/* parquet-format Type. */
enum kpw_physical_type {
    KPW_BOOLEAN = 0, KPW_INT32 = 1, KPW_INT64 = 2, KPW_INT96 = 3,
    KPW_FLOAT = 4, KPW_DOUBLE = 5, KPW_BYTE_ARRAY = 6, KPW_FIXED_LEN_BYTE_ARRAY = 7
};

/* parquet-format CompressionCodec. */
enum kpw_codec { KPW_UNCOMPRESSED = 0, KPW_SNAPPY = 1, KPW_GZIP = 2 };   /* parquet-format CompressionCodec values */

/* parquet-format Encoding. */
enum kpw_encoding {
    KPW_ENC_PLAIN = 0, KPW_ENC_PLAIN_DICTIONARY = 2, KPW_ENC_RLE = 3, KPW_ENC_BIT_PACKED = 4,
    KPW_ENC_DELTA_BINARY_PACKED = 5, KPW_ENC_DELTA_LENGTH_BYTE_ARRAY = 6, KPW_ENC_DELTA_BYTE_ARRAY = 7,
    KPW_ENC_RLE_DICTIONARY = 8
};

/* parquet-format PageType. */
enum kpw_page_type { KPW_DATA_PAGE = 0, KPW_DICTIONARY_PAGE = 2, KPW_DATA_PAGE_V2 = 3 };

/* One top-level proto2 field = one Parquet leaf column, in descriptor (declaration)
 * order, exactly as ProtoSchemaConverter lays them out.  Only scalar, non-repeated
 * fields are on the accelerated path (enum/group/message/repeated are rejected with
 * KPW_ERR_UNSUPPORTED at create time). */
typedef struct kpw_column_desc {
    const char *name;      /* Parquet column name = proto field name */
    int32_t field_number;  /* proto field number = Parquet field_id */
    int32_t proto_type;    /* enum kpw_proto_type */
    int32_t label;         /* enum kpw_proto_label */
} kpw_column_desc;

typedef struct kpw_schema {
    const char *message_name;        /* Descriptor.getFullName() -> Parquet schema name */
    const char *proto_class;         /* value of the "parquet.proto.class" footer key (may be NULL) */
    int32_t num_columns;
    const kpw_column_desc *columns;
} kpw_schema;

/* Effective parquet-mr 1.10.1 writer properties.
 *
 * Reference defaults (KafkaProtoParquetWriter.java:452-490): block_size 128 MiB,
 * page_size 128 MiB (NOT parquet-mr's 1 MiB), codec UNCOMPRESSED.  parquet-mr
 * defaults the reference never overrides: dictionary_page_size 1 MiB, writer v1,
 * max padding 8 MiB, min/max row count for size checks 100/10000.
 *
 * enable_dictionary is the value parquet-mr ends up with.  NOTE the reference quirk:
 * ParquetFile only ever calls builder.enableDictionaryEncoding() (ParquetFile.java:48-50)
 * and the parquet-mr 1.10.1 builder already defaults to dictionary ON, so the
 * reference writes dictionaries even when its enableDictionary flag is false.  The
 * host-side ParquetFile mirror reproduces that; this field lets other hosts turn it
 * off for real. */
typedef struct kpw_props {
    int64_t block_size;            /* row-group size threshold (ParquetWriter rowGroupSize) */
    int32_t page_size;             /* page size threshold */
    int32_t dictionary_page_size;  /* max dictionary byte size before PLAIN fallback */
    int32_t enable_dictionary;     /* 0/1 (effective) */
    int32_t codec;                 /* enum kpw_codec: CompressionCodecName UNCOMPRESSED / SNAPPY / GZIP
                                      (GZIP = GzipCodec without native hadoop: one
                                      java.util.zip.GZIPOutputStream member per page) */
    int32_t writer_version;        /* 1 = PARQUET_1_0 (the only version the reference reaches);
                                      2 = PARQUET_2_0 (DataPageV2, RLE_DICTIONARY, DELTA_BINARY_PACKED /
                                      DELTA_BYTE_ARRAY fallback) behind this explicit flag */
    int32_t reserved0;
    int64_t dfs_block_size;        /* 0 = local FS (NoAlignment); >0 = HDFS PaddingAlignment */
    int64_t max_padding_size;      /* parquet-mr MAX_PADDING_SIZE_DEFAULT = 8 MiB */
} kpw_props;

/* Status codes.  No C++ exception crosses the ABI.  "retryable" mirrors what the
 * reference's tryUntilSucceeds() would retry (IOException, KafkaProtoParquetWriter.java:410-428);
 * device/format errors are deliberately non-retryable so the host does not spin forever. */
enum kpw_status {
    KPW_OK = 0,
    KPW_ERR_INVALID_ARG = -1,       /* bad handle / argument (non-retryable) */
    KPW_ERR_UNSUPPORTED = -2,       /* schema/props outside the accelerated path */
    KPW_ERR_INVALID_PROTO = -3,     /* InvalidProtocolBufferException -> IllegalStateException path
                                       (KafkaProtoParquetWriter.java:268-276) */
    KPW_ERR_IO = -4,                /* output I/O failure (retryable by the host policy) */
    KPW_ERR_DEVICE = -5,            /* HIP runtime / kernel failure (non-retryable) */
    KPW_ERR_NOMEM = -6,             /* host or device allocation failure */
    KPW_ERR_STATE = -7,             /* call after close / after an earlier fatal error */
    KPW_ERR_LIMIT = -8              /* page or value larger than Integer.MAX_VALUE (ParquetEncodingException) */
};

#define KPW_DEFAULT_BLOCK_SIZE        (128LL * 1024 * 1024)
#define KPW_DEFAULT_PAGE_SIZE_PARQUET (1024 * 1024)
#define KPW_DEFAULT_DICT_PAGE_SIZE    (1024 * 1024)
#define KPW_DEFAULT_MAX_PADDING       (8LL * 1024 * 1024)

#ifdef __cplusplus
}
#endif
#endif /* KPW_TYPES_H */
