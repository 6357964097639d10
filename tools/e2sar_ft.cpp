// e2sar_ft -- file transfer over the reference-shaped C++ API (the reference's bin/e2sar_ft).
//
// Sender (bin/e2sar_ft.cpp:146-322): every regular file on the given paths (optionally
// narrowed by extension, optionally recursing into directories) is mmapped and queued as
// ONE event with addToSendQueue; the queue callback unmaps it after its last datagram has
// left (unmapFileCallback, :163-170).  Receiver (:324-448): recvEvent(1000 ms) in a loop;
// each event is written to <path>/.<prefix>_<eventNum>_<dataId>[<ext>] through an mmap of
// the new file and renamed to its final name.  Event bytes are segmented and reassembled
// by the gfx950 kernels underneath.  Options are parsed by hand (no Boost here).
//
//   e2sar_ft -s -u URI [--ip IP] [-m MTU] [--rate GBPS] [--sockets N] [--src ID] [--dataid ID]
//            [-e EXT] [--recurse] PATH...
//   e2sar_ft -r -u URI --ip IP --port P [--threads N] [--timeout MS] [--prefix P] [-e EXT]
//            [--count N] [--duration S] -p DIR
//   e2sar_ft --loopback -p OUTDIR [send options] PATH...   both sides in one process over
//            127.0.0.1 (no load balancer, so the receiver keeps the LB header)
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "e2sar_amd/e2sar.hpp"

using namespace e2sar;
using clk = std::chrono::steady_clock;

namespace {

struct Opts {
    bool send = false, recv = false, loopback = false, recurse = false;
    std::string uri, ip = "127.0.0.1", ext = ".", prefix = "e2sar_out", outDir;
    std::vector<std::string> paths;
    size_t threads = 1, sockets = 4, count = 0;
    uint16_t mtu = 1500, port = 10000, dataId = 4321;
    uint32_t src = 1234;
    float rate = -1.0f;
    int timeoutMs = 500, duration = 0, bufsize = 3 << 20;
};

bool parse(int argc, char **argv, Opts &o)
{
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto need = [&](const char *what) -> const char * {
            if (i + 1 >= argc) {
                fprintf(stderr, "option %s needs a value\n", what);
                exit(2);
            }
            return argv[++i];
        };
        if (a == "-s" || a == "--send") o.send = true;
        else if (a == "-r" || a == "--recv") o.recv = true;
        else if (a == "--loopback") o.loopback = true;
        else if (a == "-u" || a == "--uri") o.uri = need("--uri");
        else if (a == "--ip") o.ip = need("--ip");
        else if (a == "--port") o.port = (uint16_t)atoi(need("--port"));
        else if (a == "-m" || a == "--mtu") o.mtu = (uint16_t)atoi(need("--mtu"));
        else if (a == "--rate") o.rate = (float)atof(need("--rate"));
        else if (a == "--sockets") o.sockets = strtoull(need("--sockets"), nullptr, 10);
        else if (a == "--threads") o.threads = strtoull(need("--threads"), nullptr, 10);
        else if (a == "--src") o.src = (uint32_t)strtoul(need("--src"), nullptr, 10);
        else if (a == "--dataid") o.dataId = (uint16_t)atoi(need("--dataid"));
        else if (a == "-e" || a == "--extension") o.ext = need("--extension");
        else if (a == "--prefix") o.prefix = need("--prefix");
        else if (a == "--recurse") o.recurse = true;
        else if (a == "--timeout") o.timeoutMs = atoi(need("--timeout"));
        else if (a == "--count") o.count = strtoull(need("--count"), nullptr, 10);
        else if (a == "-d" || a == "--duration") o.duration = atoi(need("--duration"));
        else if (a == "-b" || a == "--bufsize") o.bufsize = atoi(need("--bufsize"));
        else if (a == "-p" || a == "--path") {
            // receive: the output directory; send: one more input path
            if (o.recv || o.loopback) o.outDir = need("--path");
            else o.paths.push_back(need("--path"));
        } else if (!a.empty() && a[0] == '-') {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return false;
        } else {
            o.paths.push_back(a);
        }
    }
    if ((int)o.send + (int)o.recv + (int)o.loopback != 1) {
        fprintf(stderr, "exactly one of -s, -r, --loopback\n");
        return false;
    }
    if ((o.recv || o.loopback) && o.outDir.empty()) {
        fprintf(stderr, "receiving needs -p DIR (given after -r / --loopback)\n");
        return false;
    }
    if (o.uri.empty())
        o.uri = "ejfat://token@127.0.0.1:18020/lb/1?data=" + o.ip + ":" + std::to_string(o.port);
    return true;
}

bool is_regular(const std::string &p)
{
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

bool is_dir(const std::string &p)
{
    struct stat st;
    return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

// checkPath (bin/e2sar_ft.cpp:243-251): regular file, extension "." matches anything
bool wanted(const std::string &p, const std::string &ext)
{
    if (!is_regular(p)) return false;
    if (ext == ".") return true;
    return p.size() >= ext.size() && p.compare(p.size() - ext.size(), ext.size(), ext) == 0;
}

// traversePaths (:257-296): files as given, directory entries (recursively with --recurse)
void collect(const std::string &p, const Opts &o, bool top, std::vector<std::string> &out)
{
    if (wanted(p, o.ext)) {
        out.push_back(p);
        return;
    }
    if (!is_dir(p) || (!top && !o.recurse)) return;
    DIR *d = opendir(p.c_str());
    if (!d) return;
    std::vector<std::string> names;
    while (dirent *e = readdir(d)) {
        if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
        names.push_back(p + "/" + e->d_name);
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    for (auto &n : names) collect(n, o, false, out);
}

struct MappedFile {
    void *ptr;
    size_t len;
    int fd;
};

// unmapFileCallback (:163-170)
void unmapFile(std::any a)
{
    auto m = std::any_cast<MappedFile>(a);
    if (m.ptr && m.len) munmap(m.ptr, m.len);
    close(m.fd);
}

// sendFile (:175-224): mmap and queue as one event, retrying while the queue is full
bool sendFile(Segmenter &s, const std::string &path, size_t &bytes)
{
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return fprintf(stderr, "Unable to open file %s\n", path.c_str()), false;
    struct stat st;
    if (fstat(fd, &st) < 0) {
        close(fd);
        return fprintf(stderr, "Unable to stat file %s\n", path.c_str()), false;
    }
    const size_t len = (size_t)st.st_size;
    void *ptr = nullptr;
    if (len) {
        ptr = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
        if (ptr == MAP_FAILED) {
            close(fd);
            return fprintf(stderr, "Unable to mmap file %s\n", path.c_str()), false;
        }
    }
    for (;;) {
        auto r = s.addToSendQueue(static_cast<uint8_t *>(ptr), len, 0, 0, 0, &unmapFile, MappedFile{ptr, len, fd});
        if (!r.has_error()) break;
        if (r.error().code() != E2SARErrorc::MemoryError) {
            fprintf(stderr, "Unexpected error submitting file into the queue: %s\n", r.error().message().c_str());
            unmapFile(MappedFile{ptr, len, fd});
            return false;
        }
        std::this_thread::yield();
    }
    bytes += len;
    return true;
}

int sendFiles(Segmenter &s, const Opts &o, size_t &nFiles)
{
    std::vector<std::string> files;
    for (auto &p : o.paths) collect(p, o, true, files);
    auto open = s.openAndStart();
    if (open.has_error()) return fprintf(stderr, "openAndStart: %s\n", open.error().message().c_str()), 1;
    const auto t0 = clk::now();
    size_t bytes = 0;
    nFiles = 0;
    for (auto &f : files) {
        printf("Queueing file %s as event %zu\n", f.c_str(), nFiles);
        if (sendFile(s, f, bytes)) nFiles++;
    }
    s.stopThreads();                       // drains the queue (:297-298)
    const double sec = std::chrono::duration<double>(clk::now() - t0).count();
    const auto st = s.getSendStats();
    printf("Estimated goodput (Gbps): %.3f\n", bytes * 8.0 / sec / 1e9);
    printf("Completed, %llu frames sent, %llu errors\n", (unsigned long long)st.msgCnt,
           (unsigned long long)st.errCnt);
    return st.errCnt ? 1 : 0;
}

// recvFiles (:356-448): a temporary dot-file written through mmap, renamed when complete.
// Stops after o.count files (0 = no limit), after o.duration seconds, or when `stop` is set.
void recvFiles(Reassembler &r, const Opts &o, std::atomic<bool> &stop, std::atomic<size_t> &written)
{
    const mode_t mode = S_IRUSR | S_IWUSR | S_IRGRP | S_IROTH;
    const auto t0 = clk::now();
    while (!stop.load()) {
        if (o.duration && clk::now() - t0 > std::chrono::seconds(o.duration)) break;
        uint8_t *buf = nullptr;
        size_t len = 0;
        EventNum_t evt = 0;
        uint16_t did = 0;
        auto g = r.recvEvent(&buf, &len, &evt, &did, 1000);
        if (g.has_error() || g.value() == -1) continue;
        std::string name = o.prefix + "_" + std::to_string(evt) + "_" + std::to_string(did);
        if (o.ext != ".") name += o.ext;
        const std::string tmp = o.outDir + "/." + name, fin = o.outDir + "/" + name;
        const int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, mode);
        bool ok = fd >= 0 && ftruncate(fd, (off_t)len) == 0;
        if (ok && len) {
            void *out = mmap(nullptr, len, PROT_WRITE, MAP_SHARED, fd, 0);
            ok = out != MAP_FAILED;
            if (ok) {
                memcpy(out, buf, len);
                ok = munmap(out, len) == 0;
            }
        }
        if (fd >= 0) close(fd);
        delete[] buf;                       // the event buffer belongs to the caller
        if (!ok) {
            fprintf(stderr, "Unable to write output file %s, continuing\n", tmp.c_str());
            continue;
        }
        rename(tmp.c_str(), fin.c_str());
        printf("Wrote %s (%zu bytes)\n", fin.c_str(), len);
        if (++written >= o.count && o.count) break;
    }
}

}  // namespace

int main(int argc, char **argv)
{
    Opts o;
    if (!parse(argc, argv, o)) return 2;
    auto uriRes = EjfatURI::getFromString(o.uri, EjfatURI::TokenType::instance);
    if (uriRes.has_error()) return fprintf(stderr, "URI: %s\n", uriRes.error().message().c_str()), 1;
    const EjfatURI uri = uriRes.value();
    Segmenter::SegmenterFlags sflags;
    sflags.useCP = false;
    sflags.mtu = o.mtu;
    sflags.rateGbps = o.rate;
    sflags.numSendSockets = o.sockets;
    sflags.sndSocketBufSize = o.bufsize;
    Reassembler::ReassemblerFlags rflags;
    rflags.useCP = false;
    rflags.withLBHeader = o.loopback;       // back to back: nobody strips the LB header
    rflags.eventTimeout_ms = o.timeoutMs;
    rflags.rcvSocketBufSize = o.bufsize;
    try {
        if (o.send) {
            Segmenter s(uri, o.dataId, o.src, sflags);
            size_t n = 0;
            return sendFiles(s, o, n);
        }
        Reassembler r(uri, o.ip, o.port, o.threads, rflags);
        auto open = r.openAndStart();
        if (open.has_error()) return fprintf(stderr, "openAndStart: %s\n", open.error().message().c_str()), 1;
        std::atomic<bool> stop{false};
        std::atomic<size_t> written{0};
        if (o.recv) {
            recvFiles(r, o, stop, written);
            r.stopThreads();
            return 0;
        }
        // loopback: count the input files first so the receiver knows when it is done
        std::vector<std::string> files;
        for (auto &p : o.paths) collect(p, o, true, files);
        size_t nonEmpty = 0;
        for (auto &f : files) {
            struct stat st;
            if (stat(f.c_str(), &st) == 0 && st.st_size > 0) nonEmpty++;   // an empty event has no datagram
        }
        o.count = nonEmpty;
        std::thread rt([&] {
            if (nonEmpty) recvFiles(r, o, stop, written);
        });
        Segmenter s(uri, o.dataId, o.src, sflags);
        size_t sent = 0;
        const int rc = sendFiles(s, o, sent);
        // the writer stops by itself after nonEmpty files; bound the wait by the
        // reassembly timeout plus a margin
        const auto deadline = clk::now() + std::chrono::milliseconds(5000 + 2 * o.timeoutMs);
        while (clk::now() < deadline && written.load() < nonEmpty)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        stop.store(true);
        rt.join();
        r.stopThreads();
        const size_t got = written.load();
        printf("Loopback: %zu files sent, %zu written\n", sent, got);
        return (rc == 0 && got == nonEmpty) ? 0 : 3;
    } catch (const E2SARException &e) {
        fprintf(stderr, "E2SARException: %s\n", e.what());
        return 1;
    }
}
