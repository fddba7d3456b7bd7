// Batch WAV reader (host only, no GPU): the dataset side of the hot path.
//
// The reference reads one file per loop iteration with Python's wave module (load_wav,
// src/audio_processing.py:9-46, called per file by experiments/run_experiments.py:90-104); the
// host mirror's RIFF walk (src/audio_processing.py _parse_riff) is the same reader in Python.
// Here a file list is read by native threads, without the interpreter lock: dsp_wav_scan walks
// every file's RIFF chunks exactly as _parse_riff does, and dsp_wav_read puts the samples of the
// mono 8/16-bit PCM files straight into the caller's packed (pinned) int16 buffer at the offsets
// the caller chose -- no per-file arrays, no concatenation, no second copy into pinned memory.
// Every other file (stereo, other widths or tags, anything malformed) is left to the Python
// reader (kind 0), which produces its samples or the reference's error for it.
#include "dsp_audiorec.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

namespace {

uint32_t le32(const unsigned char *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; }
uint32_t le16(const unsigned char *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8; }

bool pread_all(int fd, void *dst, int64_t bytes, int64_t off)
{
    char *p = static_cast<char *>(dst);
    while (bytes > 0) {
        const ssize_t r = ::pread(fd, p, (size_t)std::min<int64_t>(bytes, 1 << 30), (off_t)off);
        if (r <= 0) return false;
        p += r;
        bytes -= r;
        off += r;
    }
    return true;
}

struct Fd {
    int fd;
    explicit Fd(const char *path) : fd(::open(path, O_RDONLY | O_CLOEXEC)) {}
    ~Fd()
    {
        if (fd >= 0) ::close(fd);
    }
};

// _parse_riff's walk: RIFF/WAVE, chunks padded to even sizes, 'fmt ' (WAVE_FORMAT_PCM, channels
// and bits nonzero) before 'data', nframes = data size // frame size, the data fully present.
// The walk is bounded by the RIFF chunk (8 + its size field) as well as by the file: the wave
// module reads every subchunk through the RIFF chunk, so a RIFF size of 0 is "not a WAVE file"
// and one that ends inside the data truncates the samples -- such files are left to it (kind 0).
void scan_one(const char *path, int32_t &kind, int64_t &nsamp, int64_t &data_off)
{
    kind = DSP_WAV_OTHER;
    nsamp = data_off = 0;
    Fd f(path);
    if (f.fd < 0) return;
    struct stat st;
    if (::fstat(f.fd, &st) != 0) return;
    const int64_t n = st.st_size;
    unsigned char h[16];
    if (n < 12 || !pread_all(f.fd, h, 12, 0) || std::memcmp(h, "RIFF", 4) || std::memcmp(h + 8, "WAVE", 4)) return;
    const int64_t riff = le32(h + 4);
    if (riff < 4) return;  // wave.open: 'not a WAVE file'
    const int64_t lim = std::min<int64_t>(n, 8 + riff);
    int64_t p = 12;
    int ch = 0, sw = 0;
    bool fmt = false;
    while (p + 8 <= lim) {
        unsigned char c[8];
        if (!pread_all(f.fd, c, 8, p)) return;
        const int64_t size = le32(c + 4), body = p + 8;
        if (!std::memcmp(c, "fmt ", 4)) {
            if (size < 16 || body + 16 > lim || !pread_all(f.fd, h, 16, body)) return;
            const uint32_t tag = le16(h), channels = le16(h + 2), bits = le16(h + 14);
            if (tag != 1 || channels == 0 || bits == 0) return;
            ch = (int)channels;
            sw = (int)((bits + 7) / 8);
            fmt = true;
        } else if (!std::memcmp(c, "data", 4)) {
            if (!fmt) return;
            const int64_t frame = (int64_t)ch * sw, nbytes = size / frame * frame;
            if (body + nbytes > lim) return;  // truncated (file or RIFF size): the wave module's own behaviour (kind 0)
            if (ch == 1 && (sw == 1 || sw == 2)) {
                kind = sw == 2 ? DSP_WAV_S16_MONO : DSP_WAV_U8_MONO;
                nsamp = nbytes / sw;
                data_off = body;
            }
            return;
        }
        p = body + size + (size & 1);
    }
}

bool read_one(const char *path, int32_t kind, int64_t nsamp, int64_t data_off, int16_t *dst)
{
    Fd f(path);
    if (f.fd < 0) return false;
    if (kind == DSP_WAV_S16_MONO) return pread_all(f.fd, dst, 2 * nsamp, data_off);  // little-endian host
    // 8-bit: (u8 - 128) mod 256, load_wav's uint8 arithmetic (src/audio_processing.py:31-34)
    std::vector<unsigned char> b((size_t)std::min<int64_t>(nsamp, 1 << 20));
    for (int64_t done = 0; done < nsamp;) {
        const int64_t m = std::min<int64_t>(nsamp - done, (int64_t)b.size());
        if (!pread_all(f.fd, b.data(), m, data_off + done)) return false;
        for (int64_t j = 0; j < m; j++) dst[done + j] = (int16_t)(b[j] ^ 0x80);
        done += m;
    }
    return true;
}

// files [0, n) in chunks of 8 over min(n_threads, n / 8 + 1) threads
template <typename F> void parallel_files(int64_t n, int n_threads, F &&fn)
{
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(n_threads, n / 8 + 1));
    std::atomic<int64_t> next(0);
    auto work = [&]() {
        for (;;) {
            const int64_t a = next.fetch_add(8);
            if (a >= n) return;
            for (int64_t i = a; i < std::min<int64_t>(a + 8, n); i++) fn(i);
        }
    };
    if (nt == 1) {
        work();
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
}

}  // namespace

extern "C" int dsp_wav_scan(const char *const *paths, int64_t n, int n_threads, int32_t *kind, int64_t *nsamp,
                            int64_t *data_off)
{
    if (n < 0 || (n > 0 && (!paths || !kind || !nsamp || !data_off)) || n_threads < 1) return DSP_ERR_ARGS;
    parallel_files(n, n_threads, [&](int64_t i) { scan_one(paths[i], kind[i], nsamp[i], data_off[i]); });
    return DSP_OK;
}

extern "C" int dsp_wav_read(const char *const *paths, int64_t n, int n_threads, int32_t *kind, const int64_t *nsamp,
                            const int64_t *data_off, const int64_t *dst_off, int16_t *dst)
{
    if (n < 0 || (n > 0 && (!paths || !kind || !nsamp || !data_off || !dst_off || !dst)) || n_threads < 1)
        return DSP_ERR_ARGS;
    parallel_files(n, n_threads, [&](int64_t i) {
        if ((kind[i] == DSP_WAV_S16_MONO || kind[i] == DSP_WAV_U8_MONO) && nsamp[i] > 0 &&
            !read_one(paths[i], kind[i], nsamp[i], data_off[i], dst + dst_off[i]))
            kind[i] = DSP_WAV_OTHER;  // changed or unreadable since the scan: the caller's reader reports it
    });
    return DSP_OK;
}
