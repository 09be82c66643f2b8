/*
 * GpuCEPStreamImpl.java -- CEPStream whose query() decides, per query, where the NFA runs.
 *
 * The reference's CEPStreamImpl.query (kint/CEPStreamImpl.java:77-95) always attaches a CEPProcessor
 * and its three stores.  This one first asks PatternIR to lower the pattern over the stream's value
 * schema (SURVEY.md §8(b)):
 *   - lowered, and some device path runs it  -> a GpuCEPProcessor over libkcep.so (every key's NFA
 *     state lives on the GPU between batches, CEP_SESSION_CARRY); the reference's three stores are
 *     attached as well, for the keys that outgrow the device and continue on the reference NFA;
 *   - an opaque lambda anywhere in the chain, no value schema, an IR no device path takes, or a
 *     pattern the reference rejects (InvalidPatternException) -> the reference CEPProcessor with its
 *     NFA / event-buffer / aggregate stores, exactly as the reference wires it.
 * Either way the returned stream carries KStream<K, Sequence<K, V>>, and the query's Ir matchers are
 * bound to the schema first (PatternIR.bind), so they also evaluate on the CPU route.
 *
 * Wiring: GpuComplexStreamsBuilder (java/com/github/fhuss/kafka/streams/cep/), the drop-in for the
 * reference's ComplexStreamsBuilder (cep/ComplexStreamsBuilder.java:31-106), returns
 *     new GpuCEPStreamImpl<>(stream, schema, options)
 * from every stream(...) overload; a stream built without a schema keeps every query on the CPU.
 *
 * NOT BUILT in this repository (no JDK or Kafka jars in the image, SURVEY.md §8c).
 */
package org.apache.kafka.streams.kstream.internals;

import com.github.fhuss.kafka.streams.cep.CEPStream;
import com.github.fhuss.kafka.streams.cep.Queried;
import com.github.fhuss.kafka.streams.cep.Sequence;
import com.github.fhuss.kafka.streams.cep.pattern.Pattern;
import com.github.fhuss.kafka.streams.cep.pattern.PatternIR;
import com.github.fhuss.kafka.streams.cep.pattern.ir.IrSchema;
import com.github.fhuss.kafka.streams.cep.processor.CEPProcessor;
import com.github.fhuss.kafka.streams.cep.processor.GpuCEPProcessor;
import com.github.fhuss.kafka.streams.cep.state.QueryStoreBuilders;
import org.apache.kafka.common.serialization.Serde;
import org.apache.kafka.streams.kstream.KStream;
import org.apache.kafka.streams.processor.ProcessorSupplier;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;

import java.util.List;
import java.util.Objects;

public class GpuCEPStreamImpl<K, V> extends AbstractStream<K> implements CEPStream<K, V> {

    private static final Logger LOG = LoggerFactory.getLogger(GpuCEPStreamImpl.class);

    /** Batching knobs of the GpuCEPProcessor (flush on size, punctuation or close). */
    public static final class GpuOptions {
        public final int batchSize;         // records per cep_push_batch
        public final int maxKeys;           // dense key ids held on the device (colder keys spill to the host)
        public final long maxKeyWords;      // general path: per-key workspace cap (0 = only the device pool)
        public GpuOptions(int batchSize, int maxKeys, long maxKeyWords) {
            this.batchSize = batchSize; this.maxKeys = maxKeys; this.maxKeyWords = maxKeyWords;
        }
        public static GpuOptions defaults() { return new GpuOptions(1 << 16, 1 << 20, 0L); }
    }

    private final IrSchema<V> schema;
    private final GpuOptions options;

    @SuppressWarnings("unchecked")
    public GpuCEPStreamImpl(final KStream<K, V> stream, final IrSchema<V> schema, final GpuOptions options) {
        super((KStreamImpl<K, V>) stream);
        this.schema = schema;
        this.options = Objects.requireNonNull(options, "options can't be null");
    }

    /** The routing decision alone (also what tests and operators log). */
    public PatternIR.Lowered lower(final Pattern<K, V> pattern) {
        if (schema == null) return null;
        PatternIR.bind(pattern, schema);
        return PatternIR.encode(pattern, schema);
    }

    @Override
    public KStream<K, Sequence<K, V>> query(final String queryName, final Pattern<K, V> pattern,
                                           final Queried<K, V> queried) {
        Objects.requireNonNull(queryName, "queryName can't be null");
        Objects.requireNonNull(pattern, "pattern can't be null");
        final String processorName = builder.newProcessorName("CEPSTREAM-QUERY-" + queryName.toUpperCase() + "-");
        final PatternIR.Lowered lowered = lower(pattern);
        if (lowered != null && lowered.gpu()) {
            final byte[] ir = lowered.ir;
            final List<String> topics = lowered.topics;
            final IrSchema<V> decoder = schema;
            final GpuOptions o = options;
            final ProcessorSupplier<K, V> gpu = () ->
                new GpuCEPProcessor<>(queryName, pattern, ir, topics, decoder, o.batchSize, o.maxKeys, o.maxKeyWords);
            builder.internalTopologyBuilder.addProcessor(processorName, gpu, this.name);
            // the reference's stores stay attached: a key that outgrows the device continues on the
            // reference CEPProcessor over them (GpuCEPProcessor.handOff)
            attachReferenceStores(processorName, queryName, pattern, queried);
            LOG.info("query {}: NFA on the GPU ({} IR bytes)", queryName, ir.length);
        } else {
            LOG.info("query {}: NFA on the reference CPU path ({})", queryName,
                     lowered == null ? "no value schema for this stream" : lowered.reason);
            attachReferenceProcessor(processorName, queryName, pattern, queried);
        }
        return new KStreamImpl<>(builder, processorName, sourceNodes, false);
    }

    /** The reference's own wiring (CEPStreamImpl.java:83-92): CEPProcessor plus its three stores. */
    private void attachReferenceProcessor(final String processorName, final String queryName,
                                          final Pattern<K, V> pattern, final Queried<K, V> queried) {
        final ProcessorSupplier<K, V> cpu = () -> new CEPProcessor<>(queryName, pattern);
        builder.internalTopologyBuilder.addProcessor(processorName, cpu, this.name);
        attachReferenceStores(processorName, queryName, pattern, queried);
    }

    private void attachReferenceStores(final String processorName, final String queryName,
                                       final Pattern<K, V> pattern, final Queried<K, V> queried) {
        final Serde<K> keys = queried == null ? null : queried.keySerde();
        final Serde<V> values = queried == null ? null : queried.valueSerde();
        final QueryStoreBuilders<K, V> stores = new QueryStoreBuilders<>(queryName, pattern);
        builder.internalTopologyBuilder.addStateStore(stores.getNFAStateStoreBuilder(keys, values), processorName);
        builder.internalTopologyBuilder.addStateStore(stores.getEventBufferStoreBuilder(keys, values), processorName);
        builder.internalTopologyBuilder.addStateStore(stores.getAggregateStateStores(), processorName);
    }
}
