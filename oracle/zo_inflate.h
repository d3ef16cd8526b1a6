/*
 * zo_inflate.h -- CPU ORACLE interface.  TEST INFRASTRUCTURE ONLY.
 * Mirrors the zlib inflate surface the reference uses
 * (src/inflate.c:186 inflateInit2_, :597 inflate, :1277 inflateEnd) with its
 * own stream struct, so it can never be confused with the product library.
 */
#ifndef ZO_INFLATE_H
#define ZO_INFLATE_H
#include <stddef.h>
#include <stdint.h>

#define ZO_OK 0
#define ZO_STREAM_END 1
#define ZO_NEED_DICT 2
#define ZO_STREAM_ERROR (-2)
#define ZO_DATA_ERROR (-3)
#define ZO_MEM_ERROR (-4)
#define ZO_BUF_ERROR (-5)

#define ZO_NO_FLUSH 0
#define ZO_FINISH 4
#define ZO_BLOCK 5
#define ZO_TREES 6

typedef struct zo_code {
  uint8_t op;
  uint8_t bits;
  uint16_t val;
} zo_code;

struct zo_state;
typedef struct zo_stream {
  const uint8_t *next_in;
  uint32_t avail_in;
  uint64_t total_in;
  uint8_t *next_out;
  uint32_t avail_out;
  uint64_t total_out;
  const char *msg;
  uint32_t adler;
  int data_type;
  struct zo_state *st;
} zo_stream;

typedef struct zo_result {
  int ret;
  int data_type;
  const char *msg;
  uint64_t total_in;
  uint64_t total_out;
  uint32_t adler;
} zo_result;

uint32_t zo_crc32(uint32_t crc, const uint8_t *p, size_t n);
uint32_t zo_adler32(uint32_t adler, const uint8_t *p, size_t n);
int zo_inflate_init2(zo_stream *z, int wbits);
int zo_inflate(zo_stream *z, int flush);
int zo_inflate_end(zo_stream *z);
size_t zo_stream_size(void);
int zo_oneshot(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t cap, int wbits,
               zo_result *res);
size_t zo_js_schedule(const uint8_t *in, size_t in_len, size_t w, int wbits, char *trace,
                      size_t trace_cap, uint8_t *out, size_t out_cap, size_t *out_len);
#endif
