/*
 * png.c -- 8-bit RGBA PNG writer for the gpu/rt compatibility mode.
 *
 * gpu/rt writes its image through libpng (gpu/rt.cpp:14-54): IHDR colour type
 * 6 (RGBA), bit depth 8, no interlace, one png_write_row per buffer row, top
 * down.  libpng is not in this image, so the container format is written
 * here: signature, IHDR, one IDAT holding the zlib stream of the filtered
 * rows (filter type 0 on every row), IEND, each chunk CRC-32'd.  The pixels
 * decode identically; the compressed bytes need not match libpng's.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "rt_internal.h"

static void put32(unsigned char *p, uint32_t v)
{
  p[0] = (unsigned char)(v >> 24);
  p[1] = (unsigned char)(v >> 16);
  p[2] = (unsigned char)(v >> 8);
  p[3] = (unsigned char)v;
}

static int chunk(FILE *f, const char type[4], const unsigned char *data, size_t n)
{
  unsigned char hdr[8];
  put32(hdr, (uint32_t)n);
  memcpy(hdr + 4, type, 4);
  uLong crc = crc32(0L, (const Bytef *)type, 4);
  /* crc32() takes a uInt length: feed the data in <= 1 GiB pieces */
  for (size_t o = 0; o < n;)
  {
    size_t k = n - o > (1u << 30) ? (1u << 30) : n - o;
    crc = crc32(crc, data + o, (uInt)k);
    o += k;
  }
  unsigned char tail[4];
  put32(tail, (uint32_t)crc);
  return fwrite(hdr, 1, 8, f) == 8 && (n == 0 || fwrite(data, 1, n, f) == n) &&
         fwrite(tail, 1, 4, f) == 4 ? 0 : -1;
}

int rt_png_write_rgba(const char *path, int width, int height, const unsigned char *rgba)
{
  if (!path || width <= 0 || height <= 0 || !rgba)
    return rt_set_error(RT_EINVAL, "rt_png_write_rgba: bad argument");
  const size_t row = (size_t)width * 4, raw_n = (row + 1) * (size_t)height;
  unsigned char *raw = malloc(raw_n);
  if (!raw)
    return rt_set_error(RT_ENOMEM, "png rows (%zu bytes)", raw_n);
  for (int y = 0; y < height; y++)
  {
    raw[(row + 1) * (size_t)y] = 0; /* filter: none */
    memcpy(raw + (row + 1) * (size_t)y + 1, rgba + row * (size_t)y, row);
  }
  uLongf zn = compressBound((uLong)raw_n);
  unsigned char *z = malloc(zn);
  if (!z)
  {
    free(raw);
    return rt_set_error(RT_ENOMEM, "png deflate buffer");
  }
  int zr = compress2(z, &zn, raw, (uLong)raw_n, Z_DEFAULT_COMPRESSION);
  free(raw);
  if (zr != Z_OK)
  {
    free(z);
    return rt_set_error(RT_EIO, "png deflate failed (%d)", zr);
  }
  FILE *f = fopen(path, "wb");
  if (!f)
  {
    free(z);
    return rt_set_error(RT_EIO, "Could not open file %s", path);
  }
  static const unsigned char sig[8] = { 137, 80, 78, 71, 13, 10, 26, 10 };
  unsigned char ihdr[13];
  put32(ihdr, (uint32_t)width);
  put32(ihdr + 4, (uint32_t)height);
  ihdr[8] = 8;  /* bit depth */
  ihdr[9] = 6;  /* RGBA */
  ihdr[10] = 0; /* deflate */
  ihdr[11] = 0; /* adaptive filtering, method 0 */
  ihdr[12] = 0; /* no interlace */
  int bad = fwrite(sig, 1, 8, f) != 8 || chunk(f, "IHDR", ihdr, 13) || chunk(f, "IDAT", z, zn) ||
            chunk(f, "IEND", NULL, 0);
  free(z);
  if (fclose(f) != 0)
    bad = 1;
  return bad ? rt_set_error(RT_EIO, "write error on %s", path) : RT_OK;
}
