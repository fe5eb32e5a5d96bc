"""Ghost-cell (halo) exchange for 1-D / 2-D decomposed fields.

Reference: ``boundary_exchange`` (mpi_stencil_gt.cc:83-122),
``boundary_exchange_x`` / ``_y`` (mpi_stencil2d_gt.cc:135-373) and the SYCL
versions (mpi_stencil2d_sycl.cc:211-375, mpi_stencil2d_sycl_oo.cc:362-515):
Irecv from both neighbours, pack, device sync, Isend, Waitall, unpack — with
buffers re-allocated on every call in the gtensor version and the whole
exchange serialised against compute.

MI355X design:
  * persistent, pre-allocated pack buffers (allocated once per field);
  * all faces of one exchange are packed by ONE fused kernel launch and
    unpacked by ONE launch (``ops.copy2d_batched``);
  * y-faces (whole rows, contiguous in memory) are sent/received in place —
    zero copy, exactly the reference's dim-1 "direct" mode;
  * transport = ``torch.distributed`` point-to-point, batched into one group
    call (``batch_isend_irecv``): RCCL over xGMI for GPU ranks (each
    neighbour pair has its own xGMI link on an MI355X node, so the 2-4 faces
    proceed in parallel), gloo for CPU ranks; or host staging through pinned
    buffers ("host", the reference's ``buf:1``/``stage_host`` mode, and the
    only choice when several ranks share one GPU since RCCL refuses that);
  * split-phase API ``start()`` / ``finish()`` so the interior update can run
    on the compute stream while pack + communication run on a dedicated
    high-priority comm stream (the reference never overlaps).

Tags follow the reference convention (mpi_stencil2d_gt.cc:186-223): a message
travelling toward the lower-coordinate neighbour uses 456, toward the
higher one 123 (+1000 for the y axis).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from gpu_mpi_tests_amd import ops
from gpu_mpi_tests_amd.parallel.decomp import CartDecomp
from .field import Field2D

TAG_LOW, TAG_HIGH, TAG_Y = 456, 123, 1000


@dataclass
class _Face:
    name: str
    peer: int
    send_view: torch.Tensor  # 2-D view into the field (interior cells)
    recv_view: torch.Tensor  # 2-D view into the field (ghost cells)
    send_tag: int
    recv_tag: int
    contiguous: bool  # whole-row face that can go zero-copy
    send_buf: torch.Tensor | None = None
    recv_buf: torch.Tensor | None = None
    send_host: torch.Tensor | None = None
    recv_host: torch.Tensor | None = None
    send_span: torch.Tensor | None = None  # 1-D contiguous span covering send_view
    recv_span: torch.Tensor | None = None


def _row_span(field: Field2D, view: torch.Tensor) -> torch.Tensor:
    """Contiguous 1-D span of storage covering a [g, nx] row-block view."""
    flat = field.storage.view(-1)
    start = view.storage_offset() - field.storage.storage_offset()
    g, n = view.shape
    length = (g - 1) * field.ld + n
    return flat[start : start + length]


class HaloExchanger:
    def __init__(self, decomp: CartDecomp, field: Field2D, staging: str = "none",
                 group=None, comm_stream: "torch.cuda.Stream | None" = None):
        if staging not in ("none", "device", "host"):
            raise ValueError(f"staging must be none|device|host, got {staging!r}")
        self.decomp, self.field, self.staging = decomp, field, staging
        self.group = group
        self.device = field.storage.device
        self.is_gpu = self.device.type == "cuda"
        if self.is_gpu and comm_stream is None:
            # high priority: the halo path is the critical path of an overlapped step
            comm_stream = torch.cuda.Stream(self.device, priority=-1)
        self.comm_stream = comm_stream
        self._works: list = []
        self._pending = False
        self._h2d_done = None  # host staging: pinned recv buffers are free again
        nb = decomp.neighbors()
        f = field
        faces: list[_Face] = []
        if f.gy > 0:
            if nb["north"] is not None:
                faces.append(_Face("north", nb["north"], f.rows(0, f.gy), f.rows(-f.gy, f.gy),
                                   TAG_LOW + TAG_Y, TAG_HIGH + TAG_Y, True))
            if nb["south"] is not None:
                faces.append(_Face("south", nb["south"], f.rows(f.ny - f.gy, f.gy),
                                   f.rows(f.ny, f.gy), TAG_HIGH + TAG_Y, TAG_LOW + TAG_Y, True))
        if f.gx > 0:
            if nb["west"] is not None:
                faces.append(_Face("west", nb["west"], f.cols(0, f.gx), f.cols(-f.gx, f.gx),
                                   TAG_LOW, TAG_HIGH, False))
            if nb["east"] is not None:
                faces.append(_Face("east", nb["east"], f.cols(f.nx - f.gx, f.gx),
                                   f.cols(f.nx, f.gx), TAG_HIGH, TAG_LOW, False))
        for fc in faces:
            packed = (not fc.contiguous) or staging != "none"
            if packed:
                fc.send_buf = torch.empty(fc.send_view.shape, dtype=f.storage.dtype, device=self.device)
                fc.recv_buf = torch.empty(fc.recv_view.shape, dtype=f.storage.dtype, device=self.device)
            else:
                fc.send_span = _row_span(f, fc.send_view)
                fc.recv_span = _row_span(f, fc.recv_view)
            if staging == "host" and self.is_gpu:
                fc.send_host = torch.empty(fc.send_view.shape, dtype=f.storage.dtype, pin_memory=True)
                fc.recv_host = torch.empty(fc.recv_view.shape, dtype=f.storage.dtype, pin_memory=True)
        self.faces = faces

    # ------------------------------------------------------------------
    @property
    def active(self) -> bool:
        return bool(self.faces)

    def bytes_per_exchange(self) -> int:
        """Bytes sent by this rank per exchange (payload only)."""
        es = self.field.storage.element_size()
        return sum(fc.send_view.numel() * es for fc in self.faces)

    def _send_tensor(self, fc: _Face) -> torch.Tensor:
        if fc.send_host is not None:
            return fc.send_host
        return fc.send_buf if fc.send_buf is not None else fc.send_span

    def _recv_tensor(self, fc: _Face) -> torch.Tensor:
        if fc.recv_host is not None:
            return fc.recv_host
        return fc.recv_buf if fc.recv_buf is not None else fc.recv_span

    def _post(self) -> None:
        p2p = []
        for fc in self.faces:
            p2p.append(dist.P2POp(dist.irecv, self._recv_tensor(fc), fc.peer, self.group, fc.recv_tag))
        for fc in self.faces:
            p2p.append(dist.P2POp(dist.isend, self._send_tensor(fc), fc.peer, self.group, fc.send_tag))
        self._works = dist.batch_isend_irecv(p2p) if p2p else []

    def start(self) -> None:
        """Pack + post all sends/receives (asynchronous w.r.t. the current stream)."""
        if not self.faces:
            return
        assert not self._pending, "start() called twice without finish()"
        self._pending = True
        pack = [(fc.send_view, fc.send_buf) for fc in self.faces if fc.send_buf is not None]
        if not self.is_gpu:
            ops.copy2d_batched(pack)
            self._post()
            return
        cur = torch.cuda.current_stream(self.device)
        cs = self.comm_stream
        cs.wait_stream(cur)  # the interior cells we send were produced on `cur`
        with torch.cuda.stream(cs):
            ops.copy2d_batched(pack)
            if self.staging == "host":
                if self._h2d_done is not None:
                    self._h2d_done.synchronize()  # previous H2D from recv_host finished
                for fc in self.faces:
                    fc.send_host.copy_(fc.send_buf, non_blocking=True)
                cs.synchronize()  # host transport reads the pinned buffers
                self._post()
            else:
                self._post()

    def finish(self) -> None:
        """Wait for the exchange; on return the ghosts are valid in stream order
        of the current stream."""
        if not self.faces:
            return
        assert self._pending, "finish() without start()"
        self._pending = False
        for w in self._works:
            w.wait()  # GPU: makes the *current* stream wait on the RCCL kernels
        self._works = []
        unpack = []
        for fc in self.faces:
            if fc.recv_buf is None:
                continue
            if fc.recv_host is not None:
                fc.recv_buf.copy_(fc.recv_host, non_blocking=True)
            unpack.append((fc.recv_buf, fc.recv_view))
        if self.is_gpu and self.staging == "host":
            if self._h2d_done is None:
                self._h2d_done = torch.cuda.Event()
            self._h2d_done.record(torch.cuda.current_stream(self.device))
        ops.copy2d_batched(unpack)

    def exchange(self) -> None:
        self.start()
        self.finish()
