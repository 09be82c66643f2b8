/*
 * GpuComplexStreamsBuilder.java -- the entry point that hands out GPU-routed CEP streams, so that no
 * reference file needs an edit.
 *
 * Same surface as the reference's ComplexStreamsBuilder
 * (core/src/main/java/com/github/fhuss/kafka/streams/cep/ComplexStreamsBuilder.java:31-106): the two
 * constructors, stream(...) from a topic / topics / KStream, and build().  Every stream(...) overload
 * takes one more, optional, argument: the IrSchema that names the record value's typed columns
 * (pattern/ir/IrSchema.java).  With it, CEPStream.query() lowers the pattern to the device IR
 * (PatternIR.encode) and runs the NFA on the GPU through GpuCEPProcessor when a device path takes it;
 * without it -- the reference's own overloads, kept as they are -- every query stays on the reference
 * CEPProcessor, exactly as ComplexStreamsBuilder wires it.  GpuCEPStreamImpl.query makes that decision
 * per query (opaque lambdas, unsupported shapes and InvalidPatternException keep the CPU path).
 *
 * Migration for a user of the reference: replace `new ComplexStreamsBuilder(...)` with
 * `new GpuComplexStreamsBuilder(...)` and pass the value schema to stream(...):
 *
 *     GpuComplexStreamsBuilder builder = new GpuComplexStreamsBuilder();
 *     CEPStream<String, StockEvent> stream = builder.stream("stocks", StockIrSchema.INSTANCE);
 *     KStream<String, Sequence<String, StockEvent>> out = stream.query("Stocks", pattern, queried);
 *
 * NOT BUILT in this repository (no JDK or Kafka jars in the image, SURVEY.md §8c); its shape is
 * checked against the reference class by tests/test_patternir_cpu.py.
 */
package com.github.fhuss.kafka.streams.cep;

import com.github.fhuss.kafka.streams.cep.pattern.ir.IrSchema;
import org.apache.kafka.streams.Consumed;
import org.apache.kafka.streams.StreamsBuilder;
import org.apache.kafka.streams.Topology;
import org.apache.kafka.streams.kstream.KStream;
import org.apache.kafka.streams.kstream.internals.GpuCEPStreamImpl;
import org.apache.kafka.streams.kstream.internals.GpuCEPStreamImpl.GpuOptions;

import java.util.Collection;
import java.util.Collections;
import java.util.Objects;

public class GpuComplexStreamsBuilder {

    private final StreamsBuilder streams;
    private final GpuOptions options;

    /** Over a fresh StreamsBuilder, with the default batching (GpuOptions.defaults()). */
    public GpuComplexStreamsBuilder() {
        this(new StreamsBuilder(), GpuOptions.defaults());
    }

    /** Over the caller's StreamsBuilder (ComplexStreamsBuilder(StreamsBuilder), :48-50). */
    public GpuComplexStreamsBuilder(final StreamsBuilder builder) {
        this(builder, GpuOptions.defaults());
    }

    /** Over the caller's StreamsBuilder, with the GpuCEPProcessor's batch size / key capacity / per-key cap. */
    public GpuComplexStreamsBuilder(final StreamsBuilder builder, final GpuOptions options) {
        this.streams = Objects.requireNonNull(builder, "builder can't be null");
        this.options = Objects.requireNonNull(options, "options can't be null");
    }

    // ---- the reference's overloads: no value schema, so every query keeps the reference CPU path ----

    public <K, V> CEPStream<K, V> stream(final Collection<String> topics, final Consumed<K, V> consumed) {
        return stream(topics, consumed, null);
    }

    public <K, V> CEPStream<K, V> stream(final String topic, final Consumed<K, V> consumed) {
        return stream(topic, consumed, null);
    }

    public <K, V> CEPStream<K, V> stream(final String topic) {
        return stream(topic, (IrSchema<V>) null);
    }

    public <K, V> CEPStream<K, V> stream(final KStream<K, V> stream) {
        return stream(stream, (IrSchema<V>) null);
    }

    // ---- with the value schema: queries the device can run go to the GPU ----

    /** StreamsBuilder.stream(topics, consumed), values decoded by `schema` for the device. */
    public <K, V> CEPStream<K, V> stream(final Collection<String> topics, final Consumed<K, V> consumed,
                                         final IrSchema<V> schema) {
        return stream(streams.stream(topics, consumed), schema);
    }

    /** StreamsBuilder.stream(topic, consumed), values decoded by `schema` for the device. */
    public <K, V> CEPStream<K, V> stream(final String topic, final Consumed<K, V> consumed, final IrSchema<V> schema) {
        return stream(streams.stream(Collections.singleton(topic), consumed), schema);
    }

    /** StreamsBuilder.stream(topic), values decoded by `schema` for the device. */
    public <K, V> CEPStream<K, V> stream(final String topic, final IrSchema<V> schema) {
        final KStream<K, V> source = streams.stream(Collections.singleton(topic));
        return stream(source, schema);
    }

    /** An existing KStream as a CEPStream whose queries choose the GPU or the reference per query. */
    public <K, V> CEPStream<K, V> stream(final KStream<K, V> stream, final IrSchema<V> schema) {
        return new GpuCEPStreamImpl<>(stream, schema, options);
    }

    public Topology build() {
        return streams.build();
    }
}
