/*
 * IrSchema.java -- the typed value columns a query's records are decoded into (struct-of-arrays on the
 * GPU) and the topics its patterns name.  The Java twin of kcep/pattern.py Schema + kcep/ingest.py
 * ColumnDecoder: Expr.value() / Expr.field(name) resolve against it, PatternIR lowers with it, and
 * GpuCEPProcessor uses it as its ValueDecoder.
 *
 *   IrSchema<StockEvent> s = IrSchema.<StockEvent>builder()
 *       .longField("price", e -> e.price).longField("volume", e -> e.volume)
 *       .topics("stock-events").build();
 *   IrSchema<Integer> letters = IrSchema.ofInt();        // KStream<String, Integer>: Expr.value()
 *
 * NOT BUILT in this repository (no JDK in the image, SURVEY.md §8c).
 */
package com.github.fhuss.kafka.streams.cep.pattern.ir;

import com.github.fhuss.kafka.streams.cep.processor.GpuCEPProcessor;

import java.util.ArrayList;
import java.util.Arrays;
import java.util.Collections;
import java.util.List;
import java.util.function.ToDoubleFunction;
import java.util.function.ToLongFunction;

public final class IrSchema<V> implements GpuCEPProcessor.ValueDecoder<V> {

    private final List<String> names;
    private final int[] types;
    private final List<ToLongFunction<V>> longs;
    private final List<ToDoubleFunction<V>> doubles;
    private final List<String> topics;

    private IrSchema(Builder<V> b) {
        this.names = Collections.unmodifiableList(new ArrayList<>(b.names));
        this.types = b.types.stream().mapToInt(Integer::intValue).toArray();
        this.longs = new ArrayList<>(b.longs);
        this.doubles = new ArrayList<>(b.doubles);
        this.topics = Collections.unmodifiableList(new ArrayList<>(b.topics));
    }

    public static <V> Builder<V> builder() { return new Builder<>(); }

    /** a scalar int value (KStream<K, Integer>): Expr.value() is column 0 */
    public static IrSchema<Integer> ofInt() { return IrSchema.<Integer>builder().intField("value", v -> v).build(); }
    public static IrSchema<Long> ofLong() { return IrSchema.<Long>builder().longField("value", v -> v).build(); }
    public static IrSchema<Double> ofDouble() { return IrSchema.<Double>builder().doubleField("value", v -> v).build(); }

    public static final class Builder<V> {
        private final List<String> names = new ArrayList<>();
        private final List<Integer> types = new ArrayList<>();
        private final List<ToLongFunction<V>> longs = new ArrayList<>();
        private final List<ToDoubleFunction<V>> doubles = new ArrayList<>();
        private final List<String> topics = new ArrayList<>();

        /** a Java int field (narrowed with Java's (int) cast, kcep/ingest.py ColumnDecoder) */
        public Builder<V> intField(String name, ToLongFunction<V> get) { return add(name, Expr.INT, get, null); }
        public Builder<V> longField(String name, ToLongFunction<V> get) { return add(name, Expr.LONG, get, null); }
        public Builder<V> doubleField(String name, ToDoubleFunction<V> get) { return add(name, Expr.DOUBLE, null, get); }
        /** topics interned before the patterns' own (Schema(columns, topics=...)): ids in this order */
        public Builder<V> topics(String... t) { topics.addAll(Arrays.asList(t)); return this; }

        private Builder<V> add(String name, int type, ToLongFunction<V> l, ToDoubleFunction<V> d) {
            if (names.contains(name)) throw new IllegalArgumentException("duplicate column " + name);
            names.add(name);
            types.add(type);
            longs.add(l);
            doubles.add(d);
            return this;
        }

        public IrSchema<V> build() {
            if (names.isEmpty()) throw new IllegalArgumentException("a schema has at least one column");
            return new IrSchema<>(this);
        }
    }

    /** column index of a field (null: Event.value(), column 0), -1 if unknown */
    public int column(String name) { return name == null ? 0 : names.indexOf(name); }
    public List<String> columnNames() { return names; }
    public List<String> topics() { return topics; }
    public int[] columnTypes() { return types.clone(); }

    // ---- GpuCEPProcessor.ValueDecoder ----
    @Override public int columns() { return types.length; }
    @Override public int type(int column) { return types[column]; }
    @Override
    public long longField(V value, int column) {
        long v = longs.get(column).applyAsLong(value);
        return types[column] == Expr.INT ? (int) v : v;
    }
    @Override
    public double doubleField(V value, int column) {
        ToDoubleFunction<V> d = doubles.get(column);
        return d != null ? d.applyAsDouble(value) : (double) longField(value, column);
    }
}
