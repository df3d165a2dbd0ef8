/*
 * ref_sized_reads.c — TEST INFRASTRUCTURE ONLY (never part of the product).
 *
 * A driver of our own around the REFERENCE encoder function
 * encoders_encode_flac (/root/reference/src/encoders/flac.c:124-307, its
 * -DSTANDALONE form), linked from the reference's sources as they lie
 * (oracle/Makefile `_ref/flacenc_sized`).  It exists because the standalone
 * main (flac.c:1637-1803) reads stdin with fread, so every read() returns a
 * full block and the reference's explicit-frame-size path is never taken.
 *
 * Here the standalone stdin pcmreader (src/pcmconv.c:333-370) gets its
 * read() wrapped: the i-th call asks for read_sizes[i] frames instead of
 * block_size, then block_size as before.  The encoder cuts one frame per
 * read (flac.c:244-274), exactly what a Python PCMReader returning short
 * reads does to audiotools.encoders.encode_flac.  A listed 0 is an empty
 * read (end of stream).
 *
 * usage: flacenc_sized -c CH -r RATE -b BPS -B BLOCK -l LPC -P MINP -R MAXP
 *                      [-m] [-M] [-e] -S n1,n2,... OUT.flac  < le_signed.raw
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "pcmconv.h"

int encoders_encode_flac(char *filename, struct pcmreader_s *pcmreader,
                         unsigned block_size, unsigned max_lpc_order,
                         unsigned min_residual_partition_order,
                         unsigned max_residual_partition_order, int mid_side,
                         int adaptive_mid_side, int exhaustive_model_search);

static int (*inner_read)(struct pcmreader_s *, unsigned, aa_int *);
static unsigned *sizes;
static size_t n_sizes, next_size;

static int sized_read(struct pcmreader_s *r, unsigned pcm_frames, aa_int *ch)
{
    if (next_size < n_sizes)
        pcm_frames = sizes[next_size++];
    return inner_read(r, pcm_frames, ch);
}

static void parse_sizes(const char *s)
{
    size_t cap = 16;
    sizes = malloc(cap * sizeof(unsigned));
    while (*s) {
        char *end;
        unsigned long v = strtoul(s, &end, 10);
        if (end == s)
            break;
        if (n_sizes == cap)
            sizes = realloc(sizes, (cap *= 2) * sizeof(unsigned));
        sizes[n_sizes++] = (unsigned)v;
        s = *end ? end + 1 : end;
    }
}

int main(int argc, char *argv[])
{
    unsigned ch = 2, rate = 44100, bps = 16, block = 4096, lpc = 12, minp = 0, maxp = 6;
    int ms = 0, ams = 0, ex = 0, c;
    while ((c = getopt(argc, argv, "c:r:b:B:l:P:R:mMeS:")) != -1) {
        switch (c) {
        case 'c': ch = (unsigned)atoi(optarg); break;
        case 'r': rate = (unsigned)atoi(optarg); break;
        case 'b': bps = (unsigned)atoi(optarg); break;
        case 'B': block = (unsigned)atoi(optarg); break;
        case 'l': lpc = (unsigned)atoi(optarg); break;
        case 'P': minp = (unsigned)atoi(optarg); break;
        case 'R': maxp = (unsigned)atoi(optarg); break;
        case 'm': ms = 1; break;
        case 'M': ams = 1; break;
        case 'e': ex = 1; break;
        case 'S': parse_sizes(optarg); break;
        default: return 2;
        }
    }
    if (optind != argc - 1) {
        fprintf(stderr, "one output file required\n");
        return 2;
    }
    struct pcmreader_s *r = open_pcmreader(stdin, rate, ch, 0, bps, 0, 1);
    inner_read = r->read;
    r->read = sized_read;
    return encoders_encode_flac(argv[optind], r, block, lpc, minp, maxp, ms, ams, ex) ? 0 : 1;
}
