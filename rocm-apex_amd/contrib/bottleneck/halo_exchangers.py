"""Halo exchange for spatially split convolutions (reference
apex/contrib/bottleneck/bottleneck.py:218-385, which all-gathers 1-row halos with NCCL around its
cuDNN-frontend graphs; the exchanger classes follow the later upstream halo_exchangers module:
AllGather / SendRecv / NoComm variants behind one ``left_right_halo_exchange`` call).

The activation [N, C, H_local, W] of every rank of a spatial group holds consecutive H slabs.
``halo_pad`` returns [N, C, H_local + 2*halo, W] with ``halo`` rows of the neighbours on each
side (zeros at the global top / bottom), and its backward sends the halo gradients back to the
owning ranks.

Exchangers:

* ``HaloExchangerSendRecv`` (default): each rank posts ONE batched isend/irecv pair per
  neighbour.  xGMI is point-to-point (a direct link between every pair of GPUs of the node), so
  the neighbour exchange moves 2 * halo rows per rank over two links and its cost does not grow
  with the group size; an all-gather moves (group - 1) * 2 * halo rows into every rank.
* ``HaloExchangerAllGather``: one all-gather of the packed edge rows (the reference's pattern).
* ``HaloExchangerNoComm``: no communication, zero halos (single-rank debugging / ablations).
"""
import torch
import torch.distributed as dist


class HaloExchanger:
    """``left_right_halo_exchange(left_out, right_out) -> (left_in, right_in)``: ``left_out`` (our
    first rows) goes to the rank above, ``right_out`` (our last rows) to the rank below;
    ``left_in`` are the last rows of the rank above, ``right_in`` the first rows of the rank below
    (zeros at the global edges)."""

    def __init__(self, group, rank, world):
        self.group, self.rank, self.world = group, rank, world

    def _global(self, r):
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def left_right_halo_exchange(self, left_out, right_out):
        raise NotImplementedError


class HaloExchangerNoComm(HaloExchanger):
    def left_right_halo_exchange(self, left_out, right_out):
        return torch.zeros_like(left_out), torch.zeros_like(right_out)


class HaloExchangerAllGather(HaloExchanger):
    def left_right_halo_exchange(self, left_out, right_out):
        packed = torch.cat([left_out, right_out], dim=2).contiguous()
        out = [torch.empty_like(packed) for _ in range(self.world)]
        dist.all_gather(out, packed, group=self.group)
        h = left_out.size(2)
        left_in = out[self.rank - 1][:, :, h:] if self.rank > 0 else torch.zeros_like(left_out)
        right_in = out[self.rank + 1][:, :, :h] if self.rank + 1 < self.world else torch.zeros_like(right_out)
        return left_in, right_in


class HaloExchangerSendRecv(HaloExchanger):
    def left_right_halo_exchange(self, left_out, right_out):
        left_out, right_out = left_out.contiguous(), right_out.contiguous()
        left_in, right_in = torch.zeros_like(left_out), torch.zeros_like(right_out)
        ops = []
        if self.rank > 0:
            up = self._global(self.rank - 1)
            ops += [dist.P2POp(dist.isend, left_out, up, self.group), dist.P2POp(dist.irecv, left_in, up, self.group)]
        if self.rank + 1 < self.world:
            down = self._global(self.rank + 1)
            ops += [dist.P2POp(dist.isend, right_out, down, self.group),
                    dist.P2POp(dist.irecv, right_in, down, self.group)]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return left_in, right_in


EXCHANGERS = {"sendrecv": HaloExchangerSendRecv, "allgather": HaloExchangerAllGather,
              "nocomm": HaloExchangerNoComm}


def make_exchanger(kind, group, rank, world):
    if isinstance(kind, HaloExchanger):
        return kind
    return EXCHANGERS[kind or "sendrecv"](group, rank, world)


class HaloPad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, halo, ex):
        ctx.halo, ctx.ex = halo, ex
        above, below = ex.left_right_halo_exchange(x[:, :, :halo], x[:, :, -halo:])
        return torch.cat([above, x, below], dim=2)

    @staticmethod
    def backward(ctx, g):
        h, ex = ctx.halo, ctx.ex
        # g[:, :, :h] is the gradient of the rank above's bottom rows, g[:, :, -h:] of the rank
        # below's top rows: send them back; what arrives is the gradient of our own edge rows
        from_above, from_below = ex.left_right_halo_exchange(g[:, :, :h], g[:, :, -h:])
        gx = g[:, :, h:-h].clone()
        if ex.rank > 0:
            gx[:, :, :h] += from_above
        if ex.rank + 1 < ex.world:
            gx[:, :, -h:] += from_below
        return gx, None, None


def halo_pad(x, halo, group, rank, world, exchanger="sendrecv"):
    if world == 1:
        return torch.nn.functional.pad(x, (0, 0, halo, halo))
    return HaloPad.apply(x, halo, make_exchanger(exchanger, group, rank, world))
