/*
 * Ir.java -- matchers and aggregators that carry their body as an Expr.
 *
 * Each is an ordinary implementation of the reference's plug-in interfaces, so PredicateBuilder.where /
 * PatternBuilder.and / or / fold accept it unchanged (PredicateBuilder.java, PatternBuilder.java):
 *
 *   IrSimpleMatcher     implements SimpleMatcher.matches(event)              (SimpleMatcher.java:32-49)
 *   IrStatefulMatcher   implements StatefulMatcher.matches(event, states)    (StatefulMatcher.java:29-47)
 *   IrSequenceMatcher   implements SequenceMatcher.matches(event, seq, st)   (SequenceMatcher.java:16-38)
 *   IrAggregator        implements Aggregator.aggregate(k, v, curr)          (Aggregator.java:27-29)
 *
 * On the reference path (CEPProcessor) they evaluate their Expr with Java semantics; PatternIR reads
 * the Expr instead and lowers it.  Field accessors need the value schema: bind(schema) once per query
 * (GpuCEPStreamImpl does it for every Ir* object of the pattern before either path runs).
 *
 *   new QueryBuilder<String, StockEvent>()
 *       .select("stage-1").where(Ir.simple(Expr.field("volume").gt(1000L)))
 *           .fold("avg", Ir.fold(Expr.field("price")))
 *       .then().select("stage-2").zeroOrMore().skipTillNextMatch()...
 *
 * NOT BUILT in this repository (no JDK in the image, SURVEY.md §8c).
 */
package com.github.fhuss.kafka.streams.cep.pattern.ir;

import com.github.fhuss.kafka.streams.cep.Event;
import com.github.fhuss.kafka.streams.cep.Sequence;
import com.github.fhuss.kafka.streams.cep.pattern.Aggregator;
import com.github.fhuss.kafka.streams.cep.pattern.SequenceMatcher;
import com.github.fhuss.kafka.streams.cep.pattern.SimpleMatcher;
import com.github.fhuss.kafka.streams.cep.pattern.StatefulMatcher;
import com.github.fhuss.kafka.streams.cep.state.States;

public final class Ir {

    private Ir() {}

    /** Implemented by every matcher / aggregator whose body PatternIR can lower. */
    public interface Carrying {
        Expr expr();
        /** the value schema field accessors resolve against (also the one PatternIR lowers with) */
        void bind(IrSchema<?> schema);
    }

    public static <K, V> IrSimpleMatcher<K, V> simple(Expr e) { return new IrSimpleMatcher<>(e); }
    public static <K, V> IrStatefulMatcher<K, V> stateful(Expr e) { return new IrStatefulMatcher<>(e); }
    public static <K, V> IrSequenceMatcher<K, V> sequence(Expr e) { return new IrSequenceMatcher<>(e); }
    /** fold(state, Ir.fold(e)): the result boxed as e's static type */
    public static <K, V, T> IrAggregator<K, V, T> fold(Expr e) { return new IrAggregator<>(e, 0); }
    /** fold(state, Ir.fold(e, Expr.LONG)): the result boxed as the given type (Java's implicit widening) */
    public static <K, V, T> IrAggregator<K, V, T> fold(Expr e, int type) { return new IrAggregator<>(e, type); }

    abstract static class Base implements Carrying {
        final Expr e;
        IrSchema<?> schema;
        Base(Expr e) { this.e = e; }
        public Expr expr() { return e; }
        public void bind(IrSchema<?> schema) { this.schema = schema; }
        Expr.Env env() {
            if (schema == null) throw new IllegalStateException("Ir matcher used before bind(schema)");
            Expr.Env env = new Expr.Env();
            env.schema = schema;
            return env;
        }
    }

    public static final class IrSimpleMatcher<K, V> extends Base implements SimpleMatcher<K, V> {
        IrSimpleMatcher(Expr e) {
            super(e);
            if (!e.eventOnly()) throw new IllegalArgumentException("a SimpleMatcher reads only the event: use Ir.stateful");
        }
        @Override
        public boolean matches(Event<K, V> event) {
            Expr.Env env = env();
            env.event = event;
            env.value = event.value();
            env.hasEvent = true;
            return (Boolean) e.eval(env);
        }
    }

    public static final class IrStatefulMatcher<K, V> extends Base implements StatefulMatcher<K, V> {
        IrStatefulMatcher(Expr e) { super(e); }
        @Override
        public boolean matches(Event<K, V> event, States states) {
            Expr.Env env = env();
            env.event = event;
            env.value = event.value();
            env.hasEvent = true;
            env.states = states;
            return (Boolean) e.eval(env);
        }
    }

    public static final class IrSequenceMatcher<K, V> extends Base implements SequenceMatcher<K, V> {
        IrSequenceMatcher(Expr e) { super(e); }
        @Override
        public boolean matches(Event<K, V> event, Sequence<K, V> sequence, States states) {
            Expr.Env env = env();
            env.event = event;
            env.value = event.value();
            env.hasEvent = true;
            env.states = states;
            env.sequence = sequence;
            return (Boolean) e.eval(env);
        }
    }

    public static final class IrAggregator<K, V, T> extends Base implements Aggregator<K, V, T> {
        final int type;                         // 0: e's static type
        IrAggregator(Expr e, int type) {
            super(e);
            if (e.needsEvent()) throw new IllegalArgumentException("an Aggregator sees (key, value, curr) only");
            this.type = type;
        }
        public int resultType() { return type; }
        @Override
        @SuppressWarnings("unchecked")
        public T aggregate(K k, V v, T curr) {
            Expr.Env env = env();
            env.value = v;
            env.curr = curr;
            Object r = e.eval(env);
            if (type == Expr.LONG && r instanceof Integer) r = ((Integer) r).longValue();
            else if (type == Expr.DOUBLE && !(r instanceof Double)) r = ((Number) r).doubleValue();
            else if (type == Expr.INT && !(r instanceof Integer)) throw new ClassCastException("fold result is not an int");
            return (T) r;
        }
    }
}
