"""bench.py --op verify on the GPU (SURVEY §8(f) row 1 through the bench harness, and
the §8(e) verify-mode count): every synthetic datagram is built on the device and
filled by rns_tx_fill_dev, every 1009th is corrupted, and after the timed steps the
receive kernel must have rejected exactly those (a single flipped byte always changes
a one's-complement sum)."""
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config,steps", [("c2_64B", 12), ("c2_64B", 5), ("c3_1500B", 12)])
def test_bench_verify_rejects_exactly_the_corrupted(config, steps):
    """(c2 rotates 12 batches: 5 steps leave some unverified, and only the verified ones count.)"""
    line = bench.main(["--config", config, "--op", "verify", "--steps", str(steps), "--warmup", "1", "--ramp-s", "0",
                       "--traffic-json", "/nonexistent/{config}.json"])
    v = line["verify"]
    assert v["rejected_expected"] > 0
    assert v["rejected_total"] == v["rejected_expected"]
    assert v["datagrams_total"] > 0
    assert line["metric"] == bench.METRIC_VERIFY
    # packed receive arenas: the rows receive kernel; c2's 64-byte datagrams in 64-byte slots: the
    # strided receive kernel (rns_rx_verify_strided_dev)
    want = "csum_strided_rx_kernel" if config == "c2_64B" else "csum_rows_rx_kernel"
    assert line["roofline"]["kernel"].startswith(want)
    assert 0 < line["roofline"]["frac"] < 1.0
    assert line["cpu_baseline"] is None


def test_bench_verify_descriptor_form_matches():
    """--desc 64 (rns_rx_verify_dev, the class kernel) rejects the same planted corruptions."""
    line = bench.main(["--config", "c2_64B", "--op", "verify", "--desc", "64", "--steps", "12", "--warmup", "1",
                       "--ramp-s", "0", "--traffic-json", "/nonexistent/{config}.json"])
    assert line["roofline"]["kernel"].startswith("csum_mixed_kernel<RX>")
    assert line["verify"]["rejected_total"] == line["verify"]["rejected_expected"] > 0


@pytest.mark.parametrize("config", ["c2_64B", "c3_1500B"])
def test_bench_finalize_line(config):
    """bench.py --op finalize (SURVEY §8(f) row 2 through the bench harness): one
    rns_tx_fill_chain_dev launch per step over NetBuffer chains; after the timed steps the GPU's
    heads and statuses equal the C restatement of the transmit path run on a host copy, and the
    line carries the roofline and the CPU baseline of that restatement."""
    line = bench.main(["--config", config, "--op", "finalize", "--steps", "6", "--warmup", "1", "--ramp-s", "0",
                       "--cpu-seconds", "1"])
    assert line["metric"] == bench.METRIC_FINALIZE
    assert line["parity"]["bit_exact_all_ranks"] and line["parity"]["packets_checked"] > 0
    assert line["roofline"]["kernel"].startswith("csum_txrows_kernel FIN")
    assert 0 < line["roofline"]["frac"] < 1.0
    cb = line["cpu_baseline"]
    assert cb["gpu_sample_bit_exact"] and cb["value"] > 0 and cb["kind"] == "port"
