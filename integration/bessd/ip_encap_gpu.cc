// ip_encap_gpu.cc -- IPEncap on MI355X: the bessd module `IPEncap` replaced by a
// plugin of the same class name, gates, commands table (none: ip_encap.h) and Init
// argument, forwarding to libbessgpu.so (gpu_module.h).
#include "gpu_module.h"

// IPEncap reads three metadata attributes, prepends an IPv4 header and
// writes two attributes (ip_encap.cc:51-100): each packet's snbuf (packet
// object, metadata area, headroom, data; core/snbuf_layout.h) goes to the
// GPU whole, comes back with the header prepended and data_off / lengths
// moved, and the batch goes on to gate 0 as RunNextModule sends it.
class IPEncap final : public GpuModule {
 public:
  CommandResponse Init(const bess::pb::IPEncapArg &) {
    using AccessMode = bess::metadata::Attribute::AccessMode;
    AddMetadataAttr("ip_src", 4, AccessMode::kRead);  // ip_encap.cc:53-57
    AddMetadataAttr("ip_dst", 4, AccessMode::kRead);
    AddMetadataAttr("ip_proto", 1, AccessMode::kRead);
    AddMetadataAttr("ip_nexthop", 4, AccessMode::kWrite);
    AddMetadataAttr("ether_type", 2, AccessMode::kWrite);
    return CommandSuccess();
  }

  void ProcessBatch(Context *ctx, bess::PacketBatch *batch) override {
    const int n = batch->cnt();
    int32_t offs[5];
    for (int a = 0; a < 5; a++) offs[a] = attr_offset(a);
    uint8_t *slots[bess::PacketBatch::kMaxBurst] = {};
    uint16_t head[bess::PacketBatch::kMaxBurst] = {}, og[bess::PacketBatch::kMaxBurst] = {};
    uint32_t len[bess::PacketBatch::kMaxBurst] = {};
    for (int i = 0; i < n; i++) {
      bess::Packet *pkt = batch->pkts()[i];
      slots[i] = reinterpret_cast<uint8_t *>(pkt);
      head[i] = (uint16_t)(SNBUF_HEADROOM_OFF + pkt->data_off());
      len[i] = pkt->total_len();
    }
    if (bg_ip_encap_host(0, slots, SNBUF_SIZE, (size_t)n, SNBUF_METADATA_OFF, offs, head,
                         len, og, nullptr) < 0) {
      for (int i = 0; i < n; i++) DropPacket(ctx, batch->pkts()[i]);
      return;
    }
    for (int i = 0; i < n; i++) {  // Packet::prepend's bookkeeping (packet.h:145-154)
      bess::Packet *pkt = batch->pkts()[i];
      const uint32_t grown = len[i] - pkt->total_len();
      pkt->set_data_off((uint16_t)(head[i] - SNBUF_HEADROOM_OFF));
      pkt->set_data_len((uint16_t)(pkt->data_len() + grown));
      pkt->set_total_len(len[i]);
    }
    RunNextModule(ctx, batch);
  }
};

ADD_MODULE(IPEncap, "ip_encap", "encapsulates packets with an IPv4 header")
