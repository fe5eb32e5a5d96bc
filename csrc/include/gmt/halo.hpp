// gmt/halo.hpp — ghost-cell exchange for column-major 2-D fields.
//
// Reference: boundary_exchange_x (dim 0, non-contiguous, packed through
// device buffers, optional host staging; mpi_stencil2d_gt.cc:135-255),
// boundary_exchange_y (dim 1, contiguous, in place or through device
// buffers; :257-373), the 1-D exchange (mpi_stencil_gt.cc:83-122) and the
// SYCL versions with persistent static buffers (mpi_stencil2d_sycl.cc:211-375,
// mpi_stencil2d_sycl_oo.cc:362-515).
//
// One class covers all of them and the 2-D Cartesian case (up to four
// neighbours): x faces ("dim 0", rows of the column-major array) are packed
// by ONE fused gfx950 kernel launch for all faces and unpacked by one; y
// faces ("dim 1", whole columns) go zero-copy unless `pack_y`.  Buffers are
// allocated once.  start()/finish() are split so a caller can overlap the
// interior update with the transfer (the reference never overlaps).
//
// Tag convention of the reference (mpi_stencil2d_gt.cc:186-223): a message
// to the lower neighbour uses 456, to the upper 123; y faces add 1000.
#pragma once

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "gmt/buffer.hpp"
#include "gmt/transport.hpp"
#include "gmt/watchdog.hpp"

namespace gmt {

struct Neighbors {
  int west = -1, east = -1;    // x / dim 0 (contiguous axis) lower / upper
  int south = -1, north = -1;  // y / dim 1 (strided axis) lower / upper
  // diagonal neighbours (corner mode): known -> one-phase exchange with four
  // gx x gy corner messages; unknown (-2) -> two-phase (y faces, then x faces
  // spanning the fresh y ghosts)
  int sw = -2, se = -2, nw = -2, ne = -2;
  bool diagonals_known() const { return sw != -2 && se != -2 && nw != -2 && ne != -2; }
};

class Halo2D {
 public:
  static constexpr int kTagLow = 456, kTagHigh = 123, kTagY = 1000;
  // corner message sent toward SW/SE/NW/NE; it arrives from the opposite side
  static constexpr int kTagSW = 2000, kTagSE = 2001, kTagNW = 2002, kTagNE = 2003;

  // field: the whole ghosted array, nrows = nx + 2*gx (contiguous), ncols = ny + 2*gy.
  // corners: diagonal ghost cells must be valid too — the temporal-blocking
  // kernels (K sweeps per exchange) read them.  With the diagonal neighbours
  // known: ONE phase — x faces over the interior rows, y faces (whole
  // columns), and a gx x gy block to each diagonal neighbour, all in one
  // transport group, packed and unpacked by one fused copy launch each (the
  // corner unpack runs after the y faces landed, so it overwrites the
  // sender's stale corner ghosts they carry).  Otherwise two phases: y faces
  // first, then x faces that include the freshly received y-ghost rows.
  Halo2D(comm::Transport& t, Span2D<double> field, int gx, int gy, Neighbors nb, bool pack_y,
         int buf_space, bool corners = false)
      : t_(t), f_(field), gx_(gx), gy_(gy), nb_(nb) {
    nx_ = f_.nrows - 2 * gx;
    ny_ = f_.ncols - 2 * gy;
    const bool corner_cells = corners && gx > 0 && gy > 0 && (nb.west >= 0 || nb.east >= 0) &&
                              (nb.south >= 0 || nb.north >= 0);
    one_phase_ = corner_cells && nb.diagonals_known();
    corners_ = corner_cells && !one_phase_;  // two-phase mode
    // x faces span the y ghosts too in two-phase corner mode, and on each y
    // side without a neighbour when corner cells matter: no diagonal fills
    // that corner, so it takes the x neighbour's fixed rows (the wrapped ones
    // on an x-periodic domain)
    const bool cx = corners && gx > 0 && gy > 0;
    const bool lo_full = corners_ || (cx && nb.south < 0), hi_full = corners_ || (cx && nb.north < 0);
    const size_t xrow0 = lo_full ? 0 : gy, xrows = ny_ + (lo_full ? gy : 0) + (hi_full ? gy : 0);
    std::vector<comm::Msg> recvs, sends;
    // x faces and corner blocks are strided: packed into device buffers by
    // one fused launch, or handed to a transport that moves blocks in place
    blocks_ = t_.takes_blocks();
    auto strided = [&](Face& fc, int peer, int send_tag, int recv_tag) {
      const size_t n = static_cast<size_t>(gx) * fc.send.ncols;
      if (blocks_) {
        sends.push_back({nullptr, n * sizeof(double), peer, send_tag,
                         {fc.send.data, static_cast<size_t>(gx), fc.send.ncols, fc.send.ld}});
        recvs.push_back({nullptr, n * sizeof(double), peer, recv_tag,
                         {fc.recv.data, static_cast<size_t>(gx), fc.recv.ncols, fc.recv.ld}});
        return;
      }
      fc.sbuf = Buffer<double>(n, buf_space);
      fc.rbuf = Buffer<double>(n, buf_space);
      sends.push_back({fc.sbuf.data(), fc.sbuf.bytes(), peer, send_tag});
      recvs.push_back({fc.rbuf.data(), fc.rbuf.bytes(), peer, recv_tag});
    };
    auto x_face = [&](int peer, size_t send_row, size_t recv_row, int send_tag, int recv_tag) {
      Face fc;
      fc.send = f_.sub(send_row, gx, xrow0, xrows);
      fc.recv = f_.sub(recv_row, gx, xrow0, xrows);
      strided(fc, peer, send_tag, recv_tag);
      xfaces_.push_back(std::move(fc));
    };
    if (gx > 0) {
      if (nb.west >= 0) x_face(nb.west, gx, 0, kTagLow, kTagHigh);
      if (nb.east >= 0) x_face(nb.east, nx_, gx + nx_, kTagHigh, kTagLow);
    }
    if (one_phase_) {
      // gx x gy blocks: send rows/cols are the interior corner, recv the ghost corner
      auto corner = [&](int peer, size_t srow, size_t scol, size_t rrow, size_t rcol, int stag,
                        int rtag) {
        if (peer < 0) return;
        Face fc;
        fc.send = f_.sub(srow, gx, scol, gy);
        fc.recv = f_.sub(rrow, gx, rcol, gy);
        strided(fc, peer, stag, rtag);
        xfaces_.push_back(std::move(fc));
      };
      const size_t lo = gx, hi = nx_, glo = 0, ghi = gx + nx_;  // rows (x)
      const size_t clo = gy, chi = ny_, gclo = 0, gchi = gy + ny_;  // cols (y)
      corner(nb.sw, lo, clo, glo, gclo, kTagSW, kTagNE);
      corner(nb.se, hi, clo, ghi, gclo, kTagSE, kTagNW);
      corner(nb.nw, lo, chi, glo, gchi, kTagNW, kTagSE);
      corner(nb.ne, hi, chi, ghi, gchi, kTagNE, kTagSW);
    }
    auto y_face = [&](int peer, size_t send_col, size_t recv_col, int send_tag, int recv_tag) {
      // whole columns: contiguous from the first row of column c to the last
      // row of column c+gy-1 (exact, so a view into a padded allocation never
      // reads or writes past the field)
      const size_t n = static_cast<size_t>(gy - 1) * f_.ld + f_.nrows;
      double* s = &f_(0, send_col);
      double* r = &f_(0, recv_col);
      if (blocks_ && one_phase_ && !t_.orders_block_receives()) {
        // the interior rows of the columns only: the corner cells come from
        // the corner blocks, which this transport may write in any order
        // with the faces
        const size_t m = nx_ * static_cast<size_t>(gy);
        sends.push_back({nullptr, m * sizeof(double), peer, send_tag + kTagY,
                         {&f_(gx, send_col), nx_, static_cast<size_t>(gy), f_.ld}});
        recvs.push_back({nullptr, m * sizeof(double), peer, recv_tag + kTagY,
                         {&f_(gx, recv_col), nx_, static_cast<size_t>(gy), f_.ld}});
      } else if (pack_y) {
        Face fc;
        fc.sbuf = Buffer<double>(n, buf_space);
        fc.rbuf = Buffer<double>(n, buf_space);
        fc.ysrc = s;
        fc.ydst = r;
        fc.ybytes = n * sizeof(double);
        sends.push_back({fc.sbuf.data(), fc.sbuf.bytes(), peer, send_tag + kTagY});
        recvs.push_back({fc.rbuf.data(), fc.rbuf.bytes(), peer, recv_tag + kTagY});
        yfaces_.push_back(std::move(fc));
      } else {
        sends.push_back({s, n * sizeof(double), peer, send_tag + kTagY});
        recvs.push_back({r, n * sizeof(double), peer, recv_tag + kTagY});
      }
    };
    if (gy > 0) {
      if (nb.south >= 0) y_face(nb.south, gy, 0, kTagLow, kTagHigh);
      if (nb.north >= 0) y_face(nb.north, ny_, gy + ny_, kTagHigh, kTagLow);
    }
    for (auto& m : sends) bytes_ += m.bytes;
    nmsg_ = sends.size();
    if (corners_) {
      // phase 1 = y faces (the messages after the x faces), phase 2 = x faces
      const size_t nxm = xfaces_.size();
      std::vector<comm::Msg> rx(recvs.begin(), recvs.begin() + nxm), sx(sends.begin(), sends.begin() + nxm);
      std::vector<comm::Msg> ry(recvs.begin() + nxm, recvs.end()), sy(sends.begin() + nxm, sends.end());
      ex_ = t_.plan(ry, sy);
      ex_x_ = t_.plan(rx, sx);
    } else if (!sends.empty() || !recvs.empty()) {
      ex_ = t_.plan(recvs, sends);
    }
  }

  bool active() const { return ex_ != nullptr; }
  bool corners() const { return corners_ || one_phase_; }
  bool one_phase() const { return one_phase_; }
  // the whole exchange is stream-ordered (capturable into a hipGraph)
  bool capturable() const {
    return (!ex_ || ex_->graph_capturable()) && (!ex_x_ || ex_x_->graph_capturable());
  }
  size_t bytes_sent() const { return bytes_; }
  // pack/unpack launches of the exchanges enqueued from now on: at most n
  // workgroups in a grid-stride loop (0 = the full grid); an exchange that
  // runs beside a pass holding nearly every CU slot gets few resident
  // workgroups instead of hundreds that trickle through the free slots
  void set_pack_wgs(int n) { pack_wgs_ = n; }
  size_t messages() const { return nmsg_; }

  // packed: optional event recorded once the send buffers are packed, just
  // before the transport launches (a caller can hold its compute launch on
  // it so the transfer kernels are dispatched first and get CUs)
  void start(gmt_stream_t s, gmt_event_t packed = nullptr) {
    if (!ex_) return;
    fault_point_exchange(t_.rank());
    if (corners_) {  // y faces complete before the x faces (with their corners) are packed
      pack_y_faces(s);
      ex_->start(s);
      ex_->wait(s);
      unpack_y_faces(s);
      pack_x_faces(s);
      if (packed) GMT_CHECK("event", gmt_rt_event_record(packed, s));
      ex_x_->start(s);
      return;
    }
    pack(s);
    if (packed) GMT_CHECK("event", gmt_rt_event_record(packed, s));
    ex_->start(s);
  }
  void finish(gmt_stream_t s) {
    if (!ex_) return;
    if (corners_) {
      ex_x_->wait(s);
      unpack_x_faces(s);
    } else {
      ex_->wait(s);
      unpack(s);
    }
    watchdog_kick("halo exchange");
  }
  // Blocking exchange, reference semantics: ghosts valid and the stream
  // drained on return.
  void exchange(gmt_stream_t s) {
    start(s);
    finish(s);
    GMT_CHECK("halo sync", gmt_rt_stream_synchronize(s));
    check();
  }
  // After a synchronisation: true unless an exchange failed without the host
  // noticing (an IPC wait that timed out, gmt/transport.hpp Exchange::ok).
  bool ok(std::string* why = nullptr) const {
    return (!ex_ || ex_->ok(why)) && (!ex_x_ || ex_x_->ok(why));
  }
  // ok() or abort the job with the reason: stale ghost cells never pass
  void check() const {
    std::string why;
    if (ok(&why)) return;
    std::printf("halo exchange failed: %s\n", why.c_str());
    abort_job(EXIT_FAILURE);
  }

 private:
  struct Face {
    Buffer<double> sbuf, rbuf;
    Span2D<double> send, recv;  // x faces
    double* ysrc = nullptr;     // packed y faces
    double* ydst = nullptr;
    size_t ybytes = 0;
  };

  void pack(gmt_stream_t s) {
    pack_x_faces(s);
    pack_y_faces(s);
  }
  void unpack(gmt_stream_t s) {
    unpack_y_faces(s);  // first: packed y faces carry stale corner ghosts
    unpack_x_faces(s);  // x faces and (one-phase mode) the corner blocks
  }
  void pack_x_faces(gmt_stream_t s) {
    if (xfaces_.empty() || blocks_) return;  // blocks: the transport reads the faces in place
    gmt_copy2d_desc d[GMT_MAX_COPY2D];
    int n = 0;
    for (auto& fc : xfaces_)
      d[n++] = {fc.send.data, fc.sbuf.data(), static_cast<int64_t>(fc.send.ld),
                static_cast<int64_t>(gx_), gx_, static_cast<int64_t>(fc.send.ncols)};
    GMT_CHECK("halo pack", gmt_copy2d_batched_wgs(n, d, sizeof(double), pack_wgs_, s));
  }
  void unpack_x_faces(gmt_stream_t s) {
    if (xfaces_.empty() || blocks_) return;  // blocks: the transport wrote the ghosts in place
    gmt_copy2d_desc d[GMT_MAX_COPY2D];
    int n = 0;
    for (auto& fc : xfaces_)
      d[n++] = {fc.rbuf.data(), fc.recv.data, static_cast<int64_t>(gx_),
                static_cast<int64_t>(fc.recv.ld), gx_, static_cast<int64_t>(fc.recv.ncols)};
    GMT_CHECK("halo unpack", gmt_copy2d_batched_wgs(n, d, sizeof(double), pack_wgs_, s));
  }
  void pack_y_faces(gmt_stream_t s) {
    for (auto& fc : yfaces_)
      GMT_CHECK("halo pack y", gmt_rt_memcpy_async(fc.sbuf.data(), fc.ysrc, fc.ybytes, s));
  }
  void unpack_y_faces(gmt_stream_t s) {
    for (auto& fc : yfaces_)
      GMT_CHECK("halo unpack y", gmt_rt_memcpy_async(fc.ydst, fc.rbuf.data(), fc.ybytes, s));
  }

  comm::Transport& t_;
  Span2D<double> f_;
  int gx_, gy_;
  size_t nx_ = 0, ny_ = 0;
  Neighbors nb_;
  std::vector<Face> xfaces_, yfaces_;
  int pack_wgs_ = 0;        // set_pack_wgs
  bool blocks_ = false;     // strided faces moved in place by the transport (Transport::takes_blocks)
  bool corners_ = false;    // two-phase corner mode
  bool one_phase_ = false;  // corner blocks to the diagonal neighbours
  std::unique_ptr<comm::Exchange> ex_;    // all faces, or the y faces in corner mode
  std::unique_ptr<comm::Exchange> ex_x_;  // x faces in corner mode
  size_t bytes_ = 0, nmsg_ = 0;
};

}  // namespace gmt
