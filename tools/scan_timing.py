"""Parse-rate probe: rocJpegAmdStreamParseDevice vs host rocJpegStreamParse (+ residency) on the C2 batch."""
import sys, time; sys.path.insert(0, '.')
import bench, rocjpeg_amd as R
bench.WORKLOADS = bench._workloads()
data = bench.make_dataset(range(1234, 1234 + 1024), procs=16)
dec = R.JpegDecoder(R.Backend.HARDWARE, 0)
dec.parse_device(data[:8])
for _ in range(2):
    t = time.perf_counter(); st, ss = dec.parse_device(data); print("device", st, time.perf_counter() - t); del ss
t = time.perf_counter(); ss = [R.JpegStream(b) for b in data]; print("host", time.perf_counter() - t)
t = time.perf_counter(); ss = [R.JpegStream(b) for b in data]; dec.streams_to_device(ss); print("host parse + StreamsToDevice", time.perf_counter() - t)
